// Optional per-kernel device timing with HIP events on the context stream (diagnostics and
// bench.py's roofline: the average launch duration of each kernel, measured live).
#ifndef LOAM_PROF_HPP
#define LOAM_PROF_HPP

#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

namespace loam {

struct Prof {
  bool on = false;
  hipStream_t st = nullptr;
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<std::string, hipEvent_t>> marks;  // (segment name ending at this event)
  size_t used = 0;
  std::map<std::string, std::pair<double, long>> acc;     // name -> (ms, launches)
  hipEvent_t next() {
    if (used == pool.size()) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      pool.push_back(e);
    }
    return pool[used++];
  }
  void begin(hipStream_t s) {
    if (!on) return;
    if (!marks.empty()) {  // fold the previous run in before its events are reused
      (void)hipEventSynchronize(marks.back().second);
      collect();
    }
    st = s;
    used = 0;
    marks.clear();
    hipEvent_t e = next();
    (void)hipEventRecord(e, st);
    marks.push_back({"", e});
  }
  // the work enqueued since the previous mark is attributed to `name`
  void mark(const char* name) {
    if (!on) return;
    hipEvent_t e = next();
    (void)hipEventRecord(e, st);
    marks.push_back({name, e});
  }
  void collect() {  // after the stream has been synchronised
    if (!on) return;
    for (size_t i = 1; i < marks.size(); ++i) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, marks[i - 1].second, marks[i].second);
      auto& a = acc[marks[i].first];
      a.first += ms;
      a.second += 1;
    }
    marks.clear();
    used = 0;
  }
  ~Prof() {
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace loam
#endif
