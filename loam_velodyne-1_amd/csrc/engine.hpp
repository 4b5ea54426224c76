// Engine-internal declarations: device buffers of a batch of sweeps / problems and the kernel
// launchers of sr.hip, od.hip, mp.hip.  Not part of the C-ABI (include/loam/loam.h).
#ifndef LOAM_ENGINE_HPP
#define LOAM_ENGINE_HPP

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>
#include <string>

#include "../../include/loam/loam.h"
#include "imu.hpp"
#include "prof.hpp"

namespace loam {

// error bits a kernel may raise (per sweep / problem); mapped to LOAM_E_* by the host
enum : int {
  ERR_CAP_RING = 1,     // a ring span / segment exceeds the per-ring LDS capacity
  ERR_CAP_ROWS = 2,     // L-M row buffer overflow
  ERR_EMPTY = 4,        // no finite input point
  ERR_CAP_MAP = 8,      // map store overflow
  ERR_CAP_STACK = 16,   // stack / FromMap capacity
  ERR_VG_BITS = 32,     // a VoxelGrid segment's voxel keys exceed the bits its sort was given
};

constexpr int kSrThreads = 512;     // ring-sort workgroup (one per sweep)
constexpr int kSelThreads = 256;    // per-ring selection workgroup
constexpr int kRingCap = 4096;      // max ring span (points) handled in LDS by one workgroup
constexpr int kBigSlots = 8;        // workgroups (scratch slots) of the global-memory selection
constexpr int kSharpPerRing = 12, kLessSharpPerRing = 120, kFlatPerRing = 24;

// Launch-shape choices of the L-M loops by batch size (P = problems of the launch).  Defaults are
// the measured best; loam_set_tuning changes them per context, so that every
// path stays reachable by the parity tests and A/B measurements need no rebuild.
struct Tuning {
  int od_small_max = 63;   // k_od_rows_small (a workgroup per (queries, stored iteration)) for P <= this
  int od_fused_max = 128;  // k_od_rows<true> (step in the last workgroup) for P <= this, else + k_od_step
                           // (round 4, in the step pipeline: 128 problems 2.19 -> 2.14 ms/step; 1024 slower)
  int mp_small_max = 4;    // k_mp_lm_small (5-NN + fit + rows + step in one launch) for P <= this
  int mp_fused_max = 1 << 20;  // the fit kernel (k_mp_nnfit<true>) adds the rows and runs
                           // the step in its last workgroup for P <= this, else k_mp_iter (round 4, with
                           // k_mp_nnfit: 128 problems 3.25 -> 3.16 ms/step fused; 1024: 15.73 -> 16.32
                           // with the register reduce-scatter, 15.31 -> 15.23 with the LDS row sums)
  int od_assoc_wg = 0;     // k_od_assoc query waves (workgroups) per problem (batches, P >= 64; 0: the query
                           // capacity / 9, i.e. 64 for VLP-16, 256 for HDL-64E)
  int fit_wg = 0;          // k_mp_nnfit workgroups per problem (0: one pass over a VLP-16 stack, two for P >= 512; <= 256)
  int graph = 0;           // loam_batch_run replays the step as a captured HIP graph
  int vg_merge = 1;        // the cubes' VoxelGrid merges an old sorted prefix with the appended tail
                           // (k_vg_merge; config 3's big cubes: 95 -> 50 us per mapping frame)
  int vg_merge_min = 12288;  // ... for segments of more than this many points
  int vg_split = 1;        // the stack VoxelGrid's big segments split into 16 key-range buckets (k_vg_split /
                           // k_vg_join) instead of k_vg_big: 2 those beyond the LDS kernels, 3 already those
                           // beyond the first (2048-point) kernel, 1 (auto) 3 for HDL-64E-sized sweeps, else 2;
                           // 0: k_vg_big
  int sr_ahead = 64;       // for P >= this (0: never), loam_batch_run enqueues the next step's scan
                           // registration one step ahead (a second buffer set, a third stream), where
                           // it overlaps this step's latency-bound odometry / mapping launches.  A
                           // throughput choice for batches of independent problems: a one-problem
                           // latency (config 2) would count the next problem's work ahead of time
                           // (round 4: 128 problems 3.04 -> 2.90 ms/step, 1024: 15.12 -> 14.96)
  int step_pipe = 64;      // for P >= this (0: never): consecutive loam_batch_run steps as a software
                           // pipeline (the odometry of a step beside the mapping of the previous one;
                           // batch_enqueue_pipe), which supersedes sr_ahead (round 4: 128 problems
                           // 2.75 -> 2.37 ms/step, 1024: 14.56 -> 14.25)
  int pipe_mp_sets = 2;    // the step pipeline's mapping: 1 one set (st4, side branches on st2), 2 two sets
                           // alternating on st4 / st2 (the next frame 1 beside this frame 2; round 4:
                           // 128 problems 2.37 -> 2.20 ms/step, 1024: 14.23 -> 14.03)
  int od_graph = 1;        // loam_chain_sweep replays the odometry's L-M launches as a captured HIP graph
  int pipe_sr_sets = 3;    // the step pipeline's SR sets (and odometry state sets): with 2, a step's scan
                           // registration waits for the mapping of the step two back, so SR, seed,
                           // odometry and mapping frame 2 of one step form a cycle over two steps; with 3
                           // the cycle spans three (round 5, 128 problems: the cycle paced every step)
  int batch_streams = 1;   // the context keeps the batch pipeline's two extra streams (0: drops them)
  int sr_ahead_at = -1;    // ... starting after this point of the current step: 0 its start, 1 the
                           // odometry seed's hashes, 2 the second mapping frame; -1: 2 for P <= 256,
                           // else 1 (round 4: 128 problems 2.91 / 2.91 / 2.82 ms/step for 0 / 1 / 2;
                           // 1024: 14.98 / 14.72 / 14.96)
  int od_sel_min = 64;     // TransformToStart of the queries as its own launch (k_od_sel) for P >= this,
                           // else inside the association wave (k_od_assoc<., true>)
  int od_win_mono = 3;     // association rounds whose ring windows on ring-monotone Last clouds take the
                           // index-range search (wave_window_mono) instead of the walks: bit 0 the
                           // first (unseeded) round, bit 1 the seeded ones (round 4, 1024 problems:
                           // k_od_assoc 2.76 -> 2.42 ms/step with both)
  int od_win_mono_min = 2; // ... for P >= this (config 3's chain, P = 1: 0.733 -> 0.743 ms/sweep with them)
  int stream_defer = 1;    // loam_chain_sweep leaves the bookkeeping only the next sweep reads to the second
                           // stream: mapping's map update (insertion, per-cube VoxelGrid, compaction) after
                           // the L-M, odometry's hash tables of the new Last clouds after TransformToEnd.
                           // The sweep's outputs are downloaded without waiting for it; the next sweep waits
                           // for it first (round 5, config 3 chain: 0.70-0.74 -> 0.62-0.65 ms/sweep with the
                           // map update).  Not the message calls: their host staging waits on the second
                           // stream, and a node graph's contexts share the process's hardware queues (the
                           // three-context pipeline measured 0.45-0.51 -> 0.77-1.13 ms/sweep with it)
  int od_persist = 1;      // one problem (streaming): the odometry L-M loop as one persistent launch
                           // (k_od_lm_stream) instead of a launch per iteration and association round
  int mp_persist = 1;      // one instance (streaming): the mapping L-M loop as one persistent launch
                           // (k_mp_lm_stream) instead of a k_mp_lm_small launch per iteration
  int od_moments_min = 64; // for P >= this (and P > od_small_max), k_od_rows keeps each query's
                           // stored rows (Q12) as fp64 moments instead of re-evaluating them every
                           // iteration: O(queries) per iteration, not bit-identical, within 1e-4 of the
                           // reference on every benched problem (round 5: config 5
                           // k_od_rows 4.50 -> 2.49 ms/step, 1024 problems 1.37 -> 1.03)
  // key = value (loam_set_tuning); false for an unknown key or a value out of range.  get: the
  // current value of a key (loam_get_tuning); false for an unknown key
  bool get(const char* key, long long* v) {
    return set(key, 0, v);
  }
  bool set(const char* key, long long v, long long* read = nullptr) {
    struct K { const char* n; int* f; long long lo, hi; };
    const K ks[] = {{"od_small_max", &od_small_max, 0, 1 << 20}, {"stream_defer", &stream_defer, 0, 1}, {"pipe_sr_sets", &pipe_sr_sets, 2, 3}, {"od_graph", &od_graph, 0, 1},
                    {"od_fused_max", &od_fused_max, 0, 1 << 20},
                    {"mp_small_max", &mp_small_max, 0, 1 << 20}, {"mp_fused_max", &mp_fused_max, 0, 1 << 20},
                    {"od_assoc_wg", &od_assoc_wg, 0, 1024}, {"fit_wg", &fit_wg, 0, 256}, {"graph", &graph, 0, 1},
                    {"vg_merge", &vg_merge, 0, 1}, {"vg_merge_min", &vg_merge_min, 0, 1 << 20}, {"vg_split", &vg_split, 0, 3},
                    {"sr_ahead", &sr_ahead, 0, 1 << 20}, {"sr_ahead_at", &sr_ahead_at, -1, 2},
                    {"step_pipe", &step_pipe, 0, 1 << 20}, {"batch_streams", &batch_streams, 0, 1},
                    {"pipe_mp_sets", &pipe_mp_sets, 1, 2}, {"od_sel_min", &od_sel_min, 1, 1 << 20},
                    {"od_win_mono", &od_win_mono, 0, 3}, {"od_win_mono_min", &od_win_mono_min, 1, 1 << 20},
                    {"od_moments_min", &od_moments_min, 1, 1 << 30}, {"od_persist", &od_persist, 0, 1},
                    {"mp_persist", &mp_persist, 0, 1}};
    for (const K& k : ks)
      if (std::strcmp(key, k.n) == 0) {
        if (read) {
          *read = *k.f;
          return true;
        }
        if (v < k.lo || v > k.hi) return false;
        *k.f = (int)v;
        return true;
      }
    return false;
  }
};

// Scan-registration buffers for S sweeps of capacity `cap` points each (index s*cap + i).
struct SrBuffers {
  int S = 0, cap = 0, R = 0;
  float4* raw = nullptr;     // input (x, y, z, *) in sensor frame, per-sweep stride cap
  int* raw_n = nullptr;
  float* tmp_ori = nullptr;
  uint8_t* tmp_sid = nullptr;
  int* tilecnt = nullptr;    // [S][ntiles][R]
  int* tileF = nullptr;      // [S][ntiles] first halfPassed flip index of each tile (tile-parallel ring sort)
  int* ring_sync = nullptr;  // the fused ring sort's tile ticket
  float* sweep_ori = nullptr;  // [S][2] startOri, endOri
  float4* full = nullptr;    // ring-sorted cloud (camera frame, intensity = ring + 0.1 relTime)
  int* n_full = nullptr;
  float* curv = nullptr;
  uint8_t* picked = nullptr;
  int* sortind = nullptr;
  int8_t* label = nullptr;
  int* ring_se = nullptr;    // [S][2R] scanStartInd / scanEndInd
  int* st_sharp = nullptr;   // [S][R][12] point indices
  int* st_lsharp = nullptr;  // [S][R][120]
  int* st_flat = nullptr;    // [S][R][24]
  float4* st_lflat = nullptr;  // [S][R][kRingCap] downsampled points
  int* st_cnt = nullptr;     // [S][R][4]
  uint16_t* st_cand = nullptr;  // [S][R][kRingCap] lessFlat candidates (ring-relative), k_sr_pick -> k_sr_ringvg
  int* st_ncand = nullptr;   // [S][R]
  float4* sharp = nullptr;   // [S][12R]
  float4* lsharp = nullptr;  // [S][120R]
  float4* flat = nullptr;    // [S][24R]
  float4* lflat = nullptr;   // [S][cap]
  int* cnt = nullptr;        // [S][4]: sharp, less_sharp, flat, less_flat
  int* err = nullptr;        // [S]
  int* sel_big = nullptr;    // [S] selection kernel that handles the sweep (0 fast, 1 4096 LDS, 2 global)
  int* sel_list = nullptr;   // [2 + 2S] the sweeps routed to k_sr_select<4096, 1> / <16, 2>: counts at [0] / [1]
                             // (zeroed by k_sr_features), sweep indices at [2, 2 + S) / [2 + S, 2 + 2S)
  int* st_loff = nullptr;    // [S][R] offset of each ring's lessFlat in the sweep's st_lflat block
  uint64_t* big_keys = nullptr;  // [kBigSlots][big_stride] ring state of the global-memory selection
  int* big_sidx = nullptr;
  int* big_cand = nullptr;
  int big_stride = 0;
  __host__ __device__ int ntiles() const { return (cap + kSrThreads - 1) / kSrThreads; }
};

struct SrParams {
  int R;
  int ring_model;
  float ring_lo, ring_hi;
  loamimu::SrQueue* imu = nullptr;  // device IMU queue of sweep 0 (streaming), nullptr = no IMU
  double time_scan = 0.0;           // timeScanCur: the sweep's stamp
};

// Device allocation of the *_alloc functions: every request goes through one DevAlloc, which
// keeps the first failure and skips later requests (their pointers stay null), so an allocator
// returns one error and its *_free releases whatever was obtained.
struct DevAlloc {
  hipError_t err = hipSuccess;
  template <class T>
  void operator()(T** p, size_t bytes) {
    *p = nullptr;
    if (err != hipSuccess) return;
    void* q = nullptr;
    err = hipMalloc(&q, bytes ? bytes : 16);
    if (err == hipSuccess) *p = (T*)q;
  }
};

// Pinned host staging for the node calls' host clouds: a caller buffer is memcpy'd into the arena
// and DMA'd from there (and the reverse for outputs), instead of a pageable hipMemcpy each.  One
// arena per context, grown on demand (after a stream sync, so no copy is in flight).
struct Staging {
  float4* buf = nullptr;
  size_t cap = 0, off = 0;
  struct Pending {
    void* dst;
    const void* src;
    size_t bytes;
  };
  Pending out[8];
  int nout = 0;
  // the context's streams: any of them may still hold DMAs from the arena, so growing it (a free
  // of the old buffer) drains all of them, not only the caller's (loam_create / set_stream_priority)
  hipStream_t streams[2] = {nullptr, nullptr};
  hipError_t reserve(size_t n, hipStream_t st) {  // room for n float4 from off
    if (off + n <= cap) return hipSuccess;
    hipError_t e = hipStreamSynchronize(st);
    for (hipStream_t s : streams)
      if (e == hipSuccess && s && s != st) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    finish();
    size_t want = (off + n) * 2;
    if (want < ((size_t)1 << 17)) want = (size_t)1 << 17;
    float4* nb = nullptr;
    e = hipHostMalloc((void**)&nb, want * sizeof(float4), hipHostMallocDefault);
    if (e != hipSuccess) return e;
    if (buf) {
      if (off) memcpy(nb, buf, off * sizeof(float4));
      (void)hipHostFree(buf);
    }
    buf = nb;
    cap = want;
    return hipSuccess;
  }
  void reset() {
    off = 0;
    nout = 0;
  }
  // caller buffer -> device (async DMA from the arena)
  hipError_t up(hipStream_t st, void* dev, const void* src, size_t n) {
    if (n == 0) return hipSuccess;
    hipError_t e = reserve(n, st);
    if (e != hipSuccess) return e;
    float4* p = buf + off;
    off += n;
    memcpy(p, src, n * sizeof(float4));
    return hipMemcpyAsync(dev, p, n * sizeof(float4), hipMemcpyHostToDevice, st);
  }
  // device -> caller buffer: DMA into the arena now, the copy to dst in finish() (after a sync)
  hipError_t down(hipStream_t st, void* dst, const void* dev, size_t n) {
    if (n == 0) return hipSuccess;
    if (nout == 8) {
      hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return e;
      finish();
    }
    hipError_t e = reserve(n, st);
    if (e != hipSuccess) return e;
    float4* p = buf + off;
    off += n;
    out[nout++] = {dst, p, n * sizeof(float4)};
    return hipMemcpyAsync(p, dev, n * sizeof(float4), hipMemcpyDeviceToHost, st);
  }
  void finish() {  // the stream has been synchronised
    for (int i = 0; i < nout; ++i) memcpy(out[i].dst, out[i].src, out[i].bytes);
    nout = 0;
  }
  void release() {
    if (buf) (void)hipHostFree(buf);
    buf = nullptr;
    cap = off = 0;
    nout = 0;
  }
};

// the thread-local message loam_last_error() returns (engine.cpp)
void set_last_error(const std::string& msg);

hipError_t sr_alloc(SrBuffers& b, int S, int cap, int R);  // on failure: freed, b empty
// S sweeps packed back to back in src (sweep s at off[s], n[s] points) into raw at stride cap
// (loam_batch_feed: one host-to-device copy per chunk of sweeps instead of one per sweep)
hipError_t sr_scatter_packed(const float4* src, const int* off, const int* n, float4* raw, int cap, int S,
                             hipStream_t st);
void sr_free(SrBuffers& b);
// runs the whole scan registration for sweeps [0, S) already in b.raw / b.raw_n
// sorted (optional): recorded once the ring sort has written the full cloud (the later kernels
// only read it), so that its download can start while the feature kernels run
void sr_launch(const SrBuffers& b, const SrParams& p, hipStream_t st, Prof* prof = nullptr,
               hipEvent_t sorted = nullptr);

}  // namespace loam

#endif
