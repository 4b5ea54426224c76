// libloam_hip: host engine behind the C-ABI of include/loam/loam.h.
//
// A context owns one HIP device, one stream and the device-resident state the four reference
// nodes keep in globals: the scan-registration delay counter, the odometry transform / Last
// clouds / their voxel hashes, and the mapping cube store.  Every entry point uploads the
// caller's host cloud(s), runs the kernels of sr.hip / od.hip / mp.hip on the context stream and
// copies the results back; nothing here computes a point on the CPU (a missing GPU or kernel
// image fails loudly with LOAM_E_HIP).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstddef>
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/loam/loam.h"
#include "engine.hpp"
#include "mp.hpp"
#include "od.hpp"
#include "pose_math.hpp"

#ifdef LOAM_PIPE_TRACE
// Diagnostic builds only (tools/build_variant.sh NAME -DLOAM_PIPE_TRACE): device timestamps of the
// step pipeline's stages (events recorded on the stage's stream), printed by loam_batch_sync as
// "step stage start_us end_us" relative to the first event, to see which hand-off paces the steps.
namespace {
struct PipeTrace {
  struct Mark { int step; const char* stage; hipEvent_t a, b; };
  std::vector<Mark> marks;
  int step = 0;
  void begin(const char* stage, hipStream_t st) {
    Mark m{step, stage, nullptr, nullptr};
    (void)hipEventCreate(&m.a);
    (void)hipEventCreate(&m.b);
    (void)hipEventRecord(m.a, st);
    marks.push_back(m);
  }
  void end(const char* stage, hipStream_t st) {
    for (auto it = marks.rbegin(); it != marks.rend(); ++it)
      if (!std::strcmp(it->stage, stage) && it->step == step) { (void)hipEventRecord(it->b, st); return; }
  }
  void dump() {
    if (marks.empty()) return;
    for (auto& m : marks) {
      float a = 0, b = 0;
      if (!m.a || !m.b) continue;
      (void)hipEventElapsedTime(&a, marks[0].a, m.a);
      (void)hipEventElapsedTime(&b, marks[0].a, m.b);
      std::fprintf(stderr, "PIPE %d %s %.1f %.1f\n", m.step, m.stage, 1e3 * a, 1e3 * b);
    }
    for (auto& m : marks) {
      if (m.a) (void)hipEventDestroy(m.a);
      if (m.b) (void)hipEventDestroy(m.b);
    }
    marks.clear();
  }
};
PipeTrace g_pt;
}  // namespace
#define PT_BEGIN(s, st) g_pt.begin(s, st)
#define PT_END(s, st) g_pt.end(s, st)
#else
#define PT_BEGIN(s, st) ((void)0)
#define PT_END(s, st) ((void)0)
#endif

using namespace loam;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return fail(LOAM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
  } while (0)

FeatView feat_view(const SrBuffers& b, int first, int step) {
  FeatView v;
  const size_t R = b.R;
  v.sharp = b.sharp + (size_t)first * kSharpPerRing * R;
  v.lsharp = b.lsharp + (size_t)first * kLessSharpPerRing * R;
  v.flat = b.flat + (size_t)first * kFlatPerRing * R;
  v.lflat = b.lflat + (size_t)first * b.cap;
  v.full = b.full + (size_t)first * b.cap;
  v.sharp_stride = (size_t)step * kSharpPerRing * R;
  v.lsharp_stride = (size_t)step * kLessSharpPerRing * R;
  v.flat_stride = (size_t)step * kFlatPerRing * R;
  v.lflat_stride = (size_t)step * b.cap;
  v.full_stride = (size_t)step * b.cap;
  v.cnt = b.cnt + (size_t)first * 4;
  v.cnt_stride = 4 * step;
  v.nfull_p = b.n_full + first;
  v.nfull_stride = step;
  return v;
}

}  // namespace

constexpr size_t kMetaBytes = 8192;  // (loam_ctx::meta)

struct loam_ctx {
  loam_config cfg;
  int device = 0;
  hipStream_t st = nullptr;
  int R = 16, cap = 40000;
  // scan registration (streaming)
  int sr_init_count = 0;
  bool sr_inited = false;
  SrBuffers sr1;        // one sweep
  SrBuffers odin;       // odometry input feature set (host topics uploaded here)
  OdBuffers od1;        // one odometry problem
  bool od_inited = false;
  int od_last = 0, od_frame_count = 1;  // frameCount = skipFrameNum (src/laserOdometry.cpp:407)
  float od_sum[6] = {0, 0, 0, 0, 0, 0};  // transformSum: the streaming path accumulates it on the host
  MpBuffers mp1;        // streaming map
  int map_frame_count = 4;    // mapFrameCount = mapFrameNum - 1 (src/laserMapping.cpp:405)
  bool surround_due = false;  // the last loam_mapping frame publishes /laser_cloud_surround
  // IMU (loam_imu): scanRegistration's queue (host master copy, uploaded per sweep) and
  // laserMapping's queue
  loamimu::SrQueue* sr_imu = nullptr;     // host
  loamimu::SrQueue* sr_imu_dev = nullptr; // device
  loamimu::MpQueue mp_imu;
  double imu_last_stamp = -1e300;
  // batch (config 4)
  int P = 0;
  SrBuffers srb;
  // tune.sr_ahead: the next step's scan registration runs one step ahead on st3, into the other of
  // two buffer sets, as soon as the step that last read that set has finished (step_done); the
  // step that consumes it waits on sr_done.  The raw sweeps are uploaded into both sets.
  SrBuffers srb2;
  hipStream_t st3 = nullptr;
  hipEvent_t sr_done = nullptr, step_done[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ahead_at = nullptr;  // the point of this step after which it may start (tune.sr_ahead_at)
  // ... followed by the next step's odometry seed (Last[0] and its hashes, into the other istate
  // set), once this step's second mapping frame begins (the odometry no longer reads Last[0])
  hipEvent_t seed_at = nullptr, seed_done = nullptr;
  bool seed_ready = false;
  // tune.step_pipe: consecutive steps overlap — the odometry of a step (st) beside the mapping of the
  // previous one (st4), the scan registration + seed of the next (st3); hand-offs by events (batch_enqueue_pipe)
  hipStream_t st4 = nullptr;
  hipEvent_t od_done = nullptr, mp1_done = nullptr, a_start = nullptr, b_last = nullptr;
  hipEvent_t mp1_read = nullptr;  // frame 1 has read Last[s] (after its k_mp_stack)
  // per SR set (slot) of the step pipeline: frame 2 of the step reading set i has read Last[e]; that
  // step's mapping is done (the set's last reader)
  hipEvent_t inputs_read[3] = {nullptr, nullptr, nullptr};
  hipEvent_t mp_done[3] = {nullptr, nullptr, nullptr};
  bool mp_done_rec[3] = {false, false, false}, inputs_read_rec[3] = {false, false, false}, b_used = false;
  // the Last buffers (OdBuffers, kOdBufs of them) of the next step: its seed's (od_s, the odometry's
  // Last) and its TransformToEnd's (od_e, frame 2's input).  The step pipeline rotates (s, e) ->
  // (3 - s - e, s), so the next seed writes the buffer no running step reads and never waits for the
  // odometry; batch_enqueue keeps them.  od_s_last: the seed buffer of the last enqueued step.
  int od_s = 0, od_e = 1, od_s_last = 0;
  bool step_done_rec[3] = {false, false, false};
  int sr_idx = 0;         // the set the next step reads
  bool sr_ready = false;  // its scan registration is already enqueued (st3, sr_done)
  int srb_last = 0;       // the set of the last enqueued step (loam_batch_download)
  // tune.pipe_sr_sets = 3: the step pipeline rotates three SR sets (and odometry state sets), so a
  // step's scan registration waits for the mapping of the step three back, not two
  SrBuffers srb3;
  SrBuffers& srbuf(int i) { return i == 2 ? srb3 : (i ? srb2 : srb); }
  int pipe_k = 0;         // pipelined steps since the last drain (their mapping sets alternate by parity)
  MpBuffers mpb2;         // the second mapping set: the step pipeline's steps alternate (mpbuf)
  MpBuffers& mpbuf(int i) { return i ? mpb2 : mpb; }
  int mp_last = 0;        // the mapping set of the last enqueued step (loam_batch_download)
  // loam_batch_feed: each pipelined step's sweeps arrive from the host through the SR set the step
  // reads (copied on st3 behind that set's previous reader, then its scan registration + seed
  // there); a fed context enqueues nothing ahead at the end of a run (the feed does)
  bool fed = false;
  float4* feed_pin[3] = {nullptr, nullptr, nullptr};  // pinned staging per SR set: the sweeps back to back
  int* feed_n[3] = {nullptr, nullptr, nullptr};       // pinned sweep sizes per SR set, [2P], then offsets [2P]
  float4* feed_dev = nullptr;                         // device staging of the packed sweeps, [2P][cap] points
  int* feed_doff = nullptr;                           // device sizes + offsets, [4P]
  hipEvent_t feed_copied[3] = {nullptr, nullptr, nullptr};
  bool feed_rec[3] = {false, false, false};
  void free_feed() {
    for (int i = 0; i < 3; ++i) {
      if (feed_rec[i]) (void)hipEventSynchronize(feed_copied[i]);
      if (feed_pin[i]) (void)hipHostFree(feed_pin[i]);
      if (feed_n[i]) (void)hipHostFree(feed_n[i]);
      feed_pin[i] = nullptr;
      feed_n[i] = nullptr;
      feed_rec[i] = false;
    }
    if (feed_dev) (void)hipFree(feed_dev);
    if (feed_doff) (void)hipFree(feed_doff);
    feed_dev = nullptr;
    feed_doff = nullptr;
  }
  void reset_ahead() {    // (after draining st3 / st4)
    sr_ready = false;
    seed_ready = false;
    for (int i = 0; i < 3; ++i) mp_done_rec[i] = inputs_read_rec[i] = false;
    b_used = false;
    sr_idx = srb_last = pipe_k = 0;
    step_done_rec[0] = step_done_rec[1] = step_done_rec[2] = false;
  }
  OdBuffers odb;
  MpBuffers mpb;
  std::vector<float4> stage;
  Staging pin;                  // pinned staging of the node calls' host clouds
  // pinned scratch (8 KB) for the node calls' host-side small values, as ints:
  //   odometry           [8..19] imu_trans, [24..27]
  //                      init-frame Last counts (downloaded), [32 ..) the host copy of the
  //                      state / istate / nlast / nfullEnd download (from xb)
  // Every other small transfer of a node call goes through k_xfer (xfer.hpp): host values in its
  // arguments, device values into xb (scan registration, odometry and mapping regions)
  char* meta = nullptr;
  XferBuf xb;          // mapped, coherent host block for k_xfer's downloads (xfer.hpp regions)
  StreamIo io() { StreamIo s; s.meta = meta; s.xb = xb; s.e0 = ev[4]; s.e1 = ev[5]; return s; }
  loam_stats stats;
  Prof prof;
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipStream_t st2 = nullptr;                 // batch: mapping frame 1 beside the odometry solve
  hipEvent_t fork = nullptr, join = nullptr, fork2 = nullptr, join2 = nullptr;
  Tuning tune;                               // launch choices by batch size (loam_set_tuning)
  int prio = 0;                              // HIP priority of the context's streams (loam_set_stream_priority)
  // tune.graph: the batch step captured once as a HIP graph (for this P / these buffers) and replayed
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  int graph_P = 0;
  void drop_graph() {
    if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
    if (graph) (void)hipGraphDestroy(graph);
    graph_exec = nullptr;
    graph = nullptr;
    graph_P = 0;
    for (int i = 0; i < 2; ++i) {
      if (od_graph_exec[i]) (void)hipGraphExecDestroy(od_graph_exec[i]);
      if (od_graph[i]) (void)hipGraphDestroy(od_graph[i]);
      od_graph_exec[i] = nullptr;
      od_graph[i] = nullptr;
    }
  }
  // tune.od_graph: the streaming odometry's L-M launches (od_solve) captured once per Last-buffer
  // parity and replayed (one host call instead of ~35 launches per frame)
  hipGraph_t od_graph[2] = {nullptr, nullptr};
  hipGraphExec_t od_graph_exec[2] = {nullptr, nullptr};
};

namespace {

int check_cloud_in(const loam_cloud_in& c, int cap) {
  if (c.count > 0 && c.data == nullptr) return fail(LOAM_E_INVAL, "cloud data is null");
  if (c.stride_bytes < 12 || c.stride_bytes % 4 != 0) return fail(LOAM_E_INVAL, "bad stride_bytes");
  if (c.count > (uint32_t)cap) return fail(LOAM_E_CAPACITY, "cloud exceeds max_points");
  return LOAM_OK;
}

// (records need not be 4-byte aligned: a PointCloud2's data follows a variable-length header in
// the message, and loam_pc2_cloud hands it over in place)
// points [i0, i1) of c into dst[i0 ..) as float4 (w is not read by the device: a 16-byte stride
// is copied as is)
void pack(const loam_cloud_in& c, float4* dst, size_t i0, size_t i1) {
  const char* base = (const char*)c.data;
  if (c.stride_bytes == 16) {
    std::memcpy(dst + i0, base + i0 * 16, (i1 - i0) * 16);
    return;
  }
  for (size_t i = i0; i < i1; ++i) {
    float q[3];
    std::memcpy(q, base + i * c.stride_bytes, sizeof(q));
    dst[i] = make_float4(q[0], q[1], q[2], 0.0f);
  }
}

// device cloud -> caller storage through the pinned arena (completed by pin.finish() after a sync)
int copy_out(hipStream_t st, Staging& pin, const float4* dev, int n, loam_cloud_out* o) {
  if (o == nullptr) return LOAM_OK;
  if ((uint32_t)n > o->capacity) {
    o->count = (uint32_t)n;
    return fail(LOAM_E_CAPACITY, "output cloud capacity too small");
  }
  o->count = (uint32_t)n;
  if (n > 0) HIP_TRY(pin.down(st, o->pts, dev, (size_t)n));
  return LOAM_OK;
}

int upload_cloud(hipStream_t st, Staging& pin, const loam_cloud_out& c, float4* dev, int cap) {
  if (c.count > (uint32_t)cap) return fail(LOAM_E_CAPACITY, "input feature cloud exceeds capacity");
  if (c.count > 0) {
    if (c.pts == nullptr) return fail(LOAM_E_INVAL, "feature cloud pts is null");
    HIP_TRY(pin.up(st, dev, c.pts, (size_t)c.count));
  }
  return LOAM_OK;
}

int sr_errors(int e) {
  if (e & ERR_EMPTY) return fail(LOAM_E_INVAL, "sweep has no finite point");
  if (e & ERR_CAP_RING) return fail(LOAM_E_CAPACITY, "a ring span exceeds the per-ring capacity");
  return LOAM_OK;
}

SrParams sr_params(const loam_ctx* c) {
  SrParams p;
  p.R = c->R;
  p.ring_model = (int)c->cfg.ring_model;
  p.ring_lo = c->cfg.ring_lo_deg;
  p.ring_hi = c->cfg.ring_hi_deg;
  return p;
}

void count_bytes(loam_stats& s) {
  // algorithmic bytes, SURVEY.md §8(d)
  s.bytes_sr = 16 * s.n_raw + 32 * s.n_ring + 16 * (s.n_sharp + s.n_less_sharp + s.n_flat + s.n_less_flat);
  s.bytes_od = 16 * s.od_assoc_points + 16 * s.od_queries + 12 * s.od_queries + 32 * s.od_rows_sum;
  s.bytes_mp = 16 * s.mp_map_points + 96 * s.mp_stack_iters + 64 * s.mp_rows_sum + 32 * s.mp_stack +
               32 * s.mp_map_valid_points;
}

}  // namespace

namespace loam {
void set_last_error(const std::string& msg) { g_err = msg; }
}  // namespace loam

extern "C" {

const char* loam_last_error(void) { return g_err.c_str(); }

void loam_config_default(loam_config* d) {
  std::memset(d, 0, sizeof(*d));
  d->n_rings = 16;
  d->ring_model = LOAM_RING_VLP16;
  d->ring_lo_deg = -24.8f;
  d->ring_hi_deg = 2.0f;
  d->system_delay = 20;
  d->max_points = 40000;
  d->od_max_iter = 25;
  d->mp_max_iter = 10;
  d->skip_frame_num = 1;
  d->map_capacity = 1u << 21;
}

int loam_create(loam_ctx** out, const loam_config* cfg, int device) {
  if (out == nullptr) return fail(LOAM_E_INVAL, "out is null");
  *out = nullptr;
  loam_config c;
  if (cfg) c = *cfg;
  else loam_config_default(&c);
  if (c.n_rings < 2 || c.n_rings > 64) return fail(LOAM_E_INVAL, "n_rings must be in [2, 64]");
  if (c.max_points < 64 || c.max_points > (1u << 22)) return fail(LOAM_E_INVAL, "bad max_points");
  if (c.od_max_iter < 1 || c.od_max_iter > 1000 || c.mp_max_iter < 1 || c.mp_max_iter > 1000)
    return fail(LOAM_E_INVAL, "bad iteration limits");
  if (c.map_capacity < 1024 || c.map_capacity > (1u << 28))
    return fail(LOAM_E_INVAL, "map_capacity must be in [1024, 2^28] points");
  if (c.skip_frame_num > (1u << 20)) return fail(LOAM_E_INVAL, "bad skip_frame_num");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(LOAM_E_HIP, "no HIP device available (the engine has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(LOAM_E_INVAL, "bad device index");
  HIP_TRY(hipSetDevice(device));
  loam_ctx* x = new loam_ctx();
  x->cfg = c;
  x->device = device;
  x->R = (int)c.n_rings;
  x->cap = (int)c.max_points;
  x->od_frame_count = (int)c.skip_frame_num;
  std::memset(&x->stats, 0, sizeof(x->stats));
  if (hipStreamCreateWithFlags(&x->st, hipStreamNonBlocking) != hipSuccess) {
    delete x;
    return fail(LOAM_E_HIP, "hipStreamCreate failed");
  }
  hipError_t he = hipSuccess;
  for (auto& e : x->ev)
    if (he == hipSuccess) he = hipEventCreate(&e);
  if (he == hipSuccess && hipStreamCreateWithFlags(&x->st2, hipStreamNonBlocking) != hipSuccess) x->st2 = nullptr;
  // the batch pipeline's streams, created here with the first two: streams take the process's
  // GPU_MAX_HW_QUEUES hardware queues in creation order, and the four created together measured
  // 2.42 ms/step at the 8-GPU share against 3.13 when st3 / st4 came with the first batch (two
  // stages then shared a queue).  A context that never runs batches drops them (tuning
  // batch_streams = 0, the node pipeline's contexts), leaving the queues to the other contexts.
  if (he == hipSuccess && hipStreamCreateWithFlags(&x->st3, hipStreamNonBlocking) != hipSuccess) x->st3 = nullptr;
  if (he == hipSuccess && hipStreamCreateWithFlags(&x->st4, hipStreamNonBlocking) != hipSuccess) x->st4 = nullptr;
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->sr_done, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->ahead_at, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->seed_at, hipEventDisableTiming);
  for (hipEvent_t* e : {&x->od_done, &x->mp1_done, &x->inputs_read[0], &x->inputs_read[1], &x->inputs_read[2],
                        &x->a_start, &x->b_last, &x->mp_done[0], &x->mp_done[1], &x->mp_done[2], &x->mp1_read})
    if (he == hipSuccess) he = hipEventCreateWithFlags(e, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->seed_done, hipEventDisableTiming);
  for (auto& e : x->step_done)
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : x->feed_copied)
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  x->pin.streams[0] = x->st;
  x->pin.streams[1] = x->st2;
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->fork, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->join, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->fork2, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&x->join2, hipEventDisableTiming);
  if (he != hipSuccess) {
    loam_destroy(x);
    return fail(LOAM_E_HIP, std::string("event creation failed: ") + hipGetErrorString(he));
  }
  if (he == hipSuccess) he = sr_alloc(x->sr1, 1, x->cap, x->R);
  if (he == hipSuccess) he = sr_alloc(x->odin, 1, x->cap, x->R);
  if (he == hipSuccess) he = od_alloc(x->od1, 1, x->R, x->cap, (int)c.od_max_iter);
  if (he == hipSuccess) he = mp_alloc(x->mp1, 1, x->R, x->cap, (int)c.map_capacity, (int)c.mp_max_iter);
  x->od1.tune = x->mp1.tune = x->tune;
  if (he == hipSuccess) he = hipMalloc(&x->sr_imu_dev, sizeof(loamimu::SrQueue));
  if (he != hipSuccess) x->sr_imu_dev = nullptr;
  if (he == hipSuccess) he = hipHostMalloc((void**)&x->meta, kMetaBytes, hipHostMallocDefault);
  if (he != hipSuccess) x->meta = nullptr;
  if (he == hipSuccess) he = hipHostMalloc((void**)&x->xb.h, kXferBytes, hipHostMallocCoherent | hipHostMallocMapped);
  if (he != hipSuccess) x->xb.h = nullptr;
  else std::memset(x->xb.h, 0, kXferBytes);  // (the deferred valid-point slots are read before written)
  if (he == hipSuccess) he = hipHostGetDevicePointer((void**)&x->xb.d, x->xb.h, 0);
  x->sr_imu = new loamimu::SrQueue();
  std::memset(x->sr_imu, 0, sizeof(loamimu::SrQueue));
  x->sr_imu->last = -1;
  std::memset(&x->mp_imu, 0, sizeof(x->mp_imu));
  x->mp_imu.last = -1;
  if (he == hipSuccess) he = hipDeviceSynchronize();
  if (he != hipSuccess) {
    loam_destroy(x);
    return fail(LOAM_E_NOMEM, std::string("device allocation failed: ") + hipGetErrorString(he));
  }
  *out = x;
  return LOAM_OK;
}

void loam_destroy(loam_ctx* x) {
  if (!x) return;
  (void)hipSetDevice(x->device);
  if (x->st) (void)hipStreamSynchronize(x->st);
  if (x->st2) (void)hipStreamSynchronize(x->st2);  // (a pipelined step's mapping set runs there)
  if (x->st3) (void)hipStreamSynchronize(x->st3);
  if (x->st4) (void)hipStreamSynchronize(x->st4);
  sr_free(x->sr1);
  sr_free(x->odin);
  od_free(x->od1);
  mp_free(x->mp1);
  sr_free(x->srb);
  sr_free(x->srb2);
  sr_free(x->srb3);
  od_free(x->odb);
  mp_free(x->mpb);
  mp_free(x->mpb2);
  x->free_feed();
  for (auto& e : x->feed_copied)
    if (e) (void)hipEventDestroy(e);
  if (x->sr_imu_dev) (void)hipFree(x->sr_imu_dev);
  if (x->meta) (void)hipHostFree(x->meta);
  if (x->xb.h) (void)hipHostFree(x->xb.h);
  x->pin.release();
  delete x->sr_imu;
  for (auto& e : x->ev)
    if (e) (void)hipEventDestroy(e);
  if (x->st2) (void)hipStreamSynchronize(x->st2);
  x->drop_graph();
  if (x->fork) (void)hipEventDestroy(x->fork);
  if (x->join) (void)hipEventDestroy(x->join);
  if (x->fork2) (void)hipEventDestroy(x->fork2);
  if (x->join2) (void)hipEventDestroy(x->join2);
  if (x->sr_done) (void)hipEventDestroy(x->sr_done);
  if (x->ahead_at) (void)hipEventDestroy(x->ahead_at);
  if (x->seed_at) (void)hipEventDestroy(x->seed_at);
  for (hipEvent_t e : {x->od_done, x->mp1_done, x->inputs_read[0], x->inputs_read[1], x->inputs_read[2], x->a_start,
                       x->b_last, x->mp_done[0], x->mp_done[1], x->mp_done[2], x->mp1_read})
    if (e) (void)hipEventDestroy(e);
  if (x->st4) (void)hipStreamDestroy(x->st4);
  if (x->seed_done) (void)hipEventDestroy(x->seed_done);
  for (auto& e : x->step_done)
    if (e) (void)hipEventDestroy(e);
  if (x->st3) (void)hipStreamDestroy(x->st3);
  if (x->st2) (void)hipStreamDestroy(x->st2);
  if (x->st) (void)hipStreamDestroy(x->st);
  delete x;
}

namespace {
// the context's streams recreated at priority prio, in loam_create's order (st, st2, st3, st4: streams take the process's
// hardware queues in creation order); the batch pipeline's two only when the context keeps them
// (tuning batch_streams).  Drains the old streams first: a failure leaves the context on them.
int remake_streams(loam_ctx* x, int prio) {
  HIP_TRY(hipStreamSynchronize(x->st));
  if (x->st2) HIP_TRY(hipStreamSynchronize(x->st2));
  if (x->st3) HIP_TRY(hipStreamSynchronize(x->st3));
  if (x->st4) HIP_TRY(hipStreamSynchronize(x->st4));
  const bool batch = x->st3 != nullptr || x->st4 != nullptr;
  hipStream_t ns[4] = {nullptr, nullptr, nullptr, nullptr};
  hipError_t he = hipSuccess;
  for (int i = 0; i < (batch ? 4 : 2) && he == hipSuccess; ++i)
    he = hipStreamCreateWithPriority(&ns[i], hipStreamNonBlocking, prio);
  if (he != hipSuccess) {
    for (hipStream_t s : ns)
      if (s) (void)hipStreamDestroy(s);
    return fail(LOAM_E_HIP, "hipStreamCreateWithPriority failed (context keeps its old streams)");
  }
  for (hipStream_t s : {x->st, x->st2, x->st3, x->st4})
    if (s) (void)hipStreamDestroy(s);
  x->st = ns[0];
  x->st2 = ns[1];
  x->st3 = ns[2];
  x->st4 = ns[3];
  x->prio = prio;
  x->reset_ahead();
  x->drop_graph();  // (captured on the old streams)
  x->pin.streams[0] = x->st;
  x->pin.streams[1] = x->st2;
  return LOAM_OK;
}
}  // namespace

int loam_set_stream_priority(loam_ctx* x, int priority) {
  if (!x) return fail(LOAM_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(x->device));
  int least = 0, greatest = 0;  // HIP: a numerically lower value is a higher priority
  HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
  return remake_streams(x, priority > 0 ? greatest : priority < 0 ? least : 0);
}

int loam_set_tuning(loam_ctx* x, const char* key, long long value) {
  if (!x || !key) return fail(LOAM_E_INVAL, "null argument");
  Tuning t = x->tune;
  if (!t.set(key, value)) return fail(LOAM_E_INVAL, std::string("unknown tuning key or value out of range: ") + key);
  // (the streams below are created on the context's device, whatever device is current)
  HIP_TRY(hipSetDevice(x->device));
  HIP_TRY(hipStreamSynchronize(x->st));
  if (x->st2) HIP_TRY(hipStreamSynchronize(x->st2));
  if (x->st3) HIP_TRY(hipStreamSynchronize(x->st3));
  if (x->st4) HIP_TRY(hipStreamSynchronize(x->st4));
  if (t.batch_streams) {
    // created before anything changes (at the context's stream priority, as
    // loam_set_stream_priority creates them): a failure leaves the context as it was
    hipStream_t n3 = x->st3, n4 = x->st4;
    if (!n3) HIP_TRY(hipStreamCreateWithPriority(&n3, hipStreamNonBlocking, x->prio));
    if (!n4) {
      const hipError_t e = hipStreamCreateWithPriority(&n4, hipStreamNonBlocking, x->prio);
      if (e != hipSuccess) {
        if (n3 != x->st3) (void)hipStreamDestroy(n3);
        return fail(LOAM_E_HIP, std::string("hipStreamCreateWithPriority: ") + hipGetErrorString(e));
      }
    }
    x->st3 = n3;
    x->st4 = n4;
  } else {  // (the batch then runs on st / st2 alone)
    if (x->st3) (void)hipStreamDestroy(x->st3);
    if (x->st4) (void)hipStreamDestroy(x->st4);
    x->st3 = x->st4 = nullptr;
  }
  x->tune = t;
  x->reset_ahead();
  x->drop_graph();  // (captured with the old choices)
  x->od1.tune = x->odb.tune = t;
  x->mp1.tune = x->mpb.tune = x->mpb2.tune = t;
  return LOAM_OK;
}

int loam_get_tuning(loam_ctx* x, const char* key, long long* value) {
  if (!x || !key || !value) return fail(LOAM_E_INVAL, "null argument");
  if (!x->tune.get(key, value)) return fail(LOAM_E_INVAL, std::string("unknown tuning key: ") + key);
  return LOAM_OK;
}

int loam_set_profiling(loam_ctx* x, int on) {
  if (!x) return fail(LOAM_E_INVAL, "null argument");
  x->prof.on = on != 0;
  x->prof.acc.clear();
  return LOAM_OK;
}

int loam_get_kernel_times(loam_ctx* x, char* buf, uint32_t cap) {
  if (!x || !buf || cap == 0) return fail(LOAM_E_INVAL, "null argument");
  std::string s;
  for (auto& kv : x->prof.acc) {
    char line[256];
    std::snprintf(line, sizeof(line), "%s %.6f %ld\n", kv.first.c_str(), kv.second.first, kv.second.second);
    s += line;
  }
  if (s.size() + 1 > cap) return fail(LOAM_E_CAPACITY, "buffer too small");
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return LOAM_OK;
}

int loam_get_stats(loam_ctx* x, loam_stats* s) {
  if (!x || !s) return fail(LOAM_E_INVAL, "null argument");
  *s = x->stats;
  return LOAM_OK;
}

}  // extern "C"

namespace {
// ------------------------------------------------------------------ scanRegistration
// The laserCloudHandler body on ctx->sr1.  out == nullptr (the device-resident chain): the topics
// stay in sr1 for the odometry that follows; cnt5 (sharp, lessSharp, flat, lessFlat, full counts)
// and imu12 (/imu_trans) are returned either way.
// pending (the chain, optional): when the sweep needs no host work between the scan registration
// and the odometry (no IMU queue, no host outputs), the call returns once the kernels and the
// counts' download are enqueued, *pending = true: cnt5 are then read after the odometry's sync
// (sr_collect), and an error the scan registration reports is returned there (the odometry
// kernels it fed are undone: od_frame)
int sr_frame(loam_ctx* x, double stamp, const loam_cloud_in& raw, loam_features* out, int* cnt5, float* imu12,
             bool* pending = nullptr) {
  if (!x->sr_inited) {  // src/scanRegistration.cpp:213-219 (Q1)
    x->sr_init_count++;
    if (x->sr_init_count >= (int)x->cfg.system_delay) x->sr_inited = true;
    return fail(LOAM_E_NOT_READY, "inside systemDelay");
  }
  int rc = check_cloud_in(raw, x->cap);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(x->device));
  SrBuffers& b = x->sr1;
  const int n = (int)raw.count;
  x->pin.reset();
  HIP_TRY(x->pin.reserve((size_t)2 * n, x->st));
  float4* praw = x->pin.buf;  // the sweep packed straight into pinned memory
  float4* pfull = x->pin.buf + n;  // the early download of the full cloud (below)
  x->pin.off = (size_t)2 * n;
  // packed in chunks, each chunk's DMA overlapping the packing of the next
  constexpr size_t kPackChunk = 8192;
  for (size_t i0 = 0; i0 < (size_t)n; i0 += kPackChunk) {
    const size_t i1 = std::min((size_t)n, i0 + kPackChunk);
    pack(raw, praw, i0, i1);
    HIP_TRY(hipMemcpyAsync(b.raw + i0, praw + i0, (i1 - i0) * sizeof(float4), hipMemcpyHostToDevice, x->st));
  }
  {
    Xfer xp;
    xp.put(b.raw_n, &n, sizeof(int));
    HIP_TRY(xfer_launch(xp, x->st));
  }
  SrParams prm = sr_params(x);
  loamimu::SrQueue* q = x->sr_imu;
  const size_t tail = offsetof(loamimu::SrQueue, front);  // pointers, Start, Cur, FromStart
  if (q->last >= 0) {  // IMU de-skew (:286-349) with the queue as loam_imu left it
    HIP_TRY(hipMemcpyAsync(x->sr_imu_dev, q, sizeof(*q), hipMemcpyHostToDevice, x->st));
    prm.imu = x->sr_imu_dev;
    prm.time_scan = stamp;
  }
  HIP_TRY(hipEventRecord(x->ev[0], x->st));
  // /velodyne_cloud_2 is final once the rings are sorted: its n (>= the kept points) points come
  // down on the second stream, and reach the caller's buffer on the host, while the curvature /
  // pick / VoxelGrid kernels run
  // (only when the caller's buffer holds all n points: nfull <= n can then not fail on capacity)
  const bool early = out && x->st2 != nullptr && n > 0 && out->full.pts && (uint32_t)n <= out->full.capacity;
  sr_launch(b, prm, x->st, nullptr, early ? x->fork : nullptr);
  HIP_TRY(hipEventRecord(x->ev[1], x->st));
  HIP_TRY(hipGetLastError());
  if (early) {
    HIP_TRY(hipStreamWaitEvent(x->st2, x->fork, 0));
    HIP_TRY(hipMemcpyAsync(pfull, b.full, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost, x->st2));
    HIP_TRY(hipEventRecord(x->join, x->st2));
  }
  if (q->last >= 0)
    HIP_TRY(hipMemcpyAsync((char*)q + tail, (const char*)x->sr_imu_dev + tail, sizeof(*q) - tail,
                           hipMemcpyDeviceToHost, x->st));
  // [1..4] counts, [5] nfull, [6] err into the mapped host block, one launch
  const int* mi = (const int*)(x->xb.h + kXferSr) - 1;
  {
    Xfer xg;
    xg.get(x->xb.d + kXferSr, b.cnt, 4 * sizeof(int));
    xg.get(x->xb.d + kXferSr + 16, b.n_full, sizeof(int));
    xg.get(x->xb.d + kXferSr + 20, b.err, sizeof(int));
    HIP_TRY(xfer_launch(xg, x->st));
  }
  HIP_TRY(hipGetLastError());
  if (pending && !out && q->last < 0) {  // (the chain: no sync here, sr_collect after the odometry)
    const float it[12] = {q->pitchStart, q->yawStart, q->rollStart, q->pitchCur, q->yawCur, q->rollCur,
                          q->shiftFSX,   q->shiftFSY, q->shiftFSZ,  q->veloFSX,  q->veloFSY, q->veloFSZ};
    std::memcpy(imu12, it, sizeof(it));
    for (int k = 0; k < 5; ++k) cnt5[k] = 0;
    *pending = true;
    return LOAM_OK;
  }
  HIP_TRY(hipStreamSynchronize(x->st));
  int cnt[4] = {mi[1], mi[2], mi[3], mi[4]};
  const int nfull = mi[5];
  rc = sr_errors(mi[6]);
  if (rc) {
    if (early) HIP_TRY(hipEventSynchronize(x->join));  // the arena is reused by the next call
    return rc;  // (nothing written to the caller's buffers)
  }
  if (early) {
    HIP_TRY(hipEventSynchronize(x->join));
    std::memcpy(out->full.pts, pfull, (size_t)nfull * sizeof(float4));
  }
  int e = 0;
  x->pin.reset();
  if (out) {
    if (early) {
      out->full.count = (uint32_t)nfull;
      if ((uint32_t)nfull > out->full.capacity) e |= fail(LOAM_E_CAPACITY, "output cloud capacity too small");
    } else {
      e |= copy_out(x->st, x->pin, b.full, nfull, &out->full);
    }
    e |= copy_out(x->st, x->pin, b.sharp, cnt[0], &out->sharp);
    e |= copy_out(x->st, x->pin, b.lsharp, cnt[1], &out->less_sharp);
    e |= copy_out(x->st, x->pin, b.flat, cnt[2], &out->flat);
    e |= copy_out(x->st, x->pin, b.lflat, cnt[3], &out->less_flat);
    HIP_TRY(hipStreamSynchronize(x->st));
    x->pin.finish();
  }
  // /imu_trans (:614-635)
  const float it[12] = {q->pitchStart, q->yawStart, q->rollStart, q->pitchCur, q->yawCur, q->rollCur,
                        q->shiftFSX,   q->shiftFSY, q->shiftFSZ,  q->veloFSX,  q->veloFSY, q->veloFSZ};
  if (out) std::memcpy(out->imu_trans, it, sizeof(it));
  std::memcpy(imu12, it, sizeof(it));
  for (int k = 0; k < 4; ++k) cnt5[k] = cnt[k];
  cnt5[4] = nfull;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, x->ev[0], x->ev[1]);
  std::memset(&x->stats, 0, sizeof(x->stats));
  x->stats.n_raw = (uint64_t)n;
  x->stats.n_ring = (uint64_t)nfull;
  x->stats.n_sharp = cnt[0]; x->stats.n_less_sharp = cnt[1];
  x->stats.n_flat = cnt[2]; x->stats.n_less_flat = cnt[3];
  x->stats.ms_sr = ms;
  count_bytes(x->stats);
  return e ? LOAM_E_CAPACITY : LOAM_OK;
}

// a pending scan registration's results (sr_frame's pending mode), once the stream has been
// synchronised past them: its error code; cnt5 filled
int sr_collect(loam_ctx* x, int* cnt5) {
  const int* mi = (const int*)(x->xb.h + kXferSr) - 1;
  for (int k = 0; k < 4; ++k) cnt5[k] = mi[1 + k];
  cnt5[4] = mi[5];
  return sr_errors(mi[6]);
}

// ------------------------------------------------------------------ laserOdometry
// The laserOdometry loop body on the features fv (cnt: sharp, lessSharp, flat, lessFlat, full
// counts; imu: /imu_trans).  late_full: the full cloud is still on the host (message mode) and is
// staged while the L-M runs; nullptr when fv's full cloud is already on the device.  nl3 (optional):
// the published CornerLast / SurfLast / full-cloud counts, for a mapping on the device copies.
int od_frame(loam_ctx* x, const FeatView& fv, const int* cnt, const float* imu, const loam_cloud_out* late_full,
             loam_pose6* sum_out, loam_cloud_out* corner_last, loam_cloud_out* surf_last, loam_cloud_out* full_end,
             int* published, int* nl3, bool defer = false, bool sr_pending = false);
}  // namespace

extern "C" {
int loam_scan_registration(loam_ctx* x, double stamp, loam_cloud_in raw, loam_features* out) {
  if (!x || !out) return fail(LOAM_E_INVAL, "null argument");
  int cnt5[5];
  float imu12[12];
  return sr_frame(x, stamp, raw, out, cnt5, imu12);
}

int loam_odometry(loam_ctx* x, double stamp, const loam_features* in, loam_pose6* sum_out,
                  loam_cloud_out* corner_last, loam_cloud_out* surf_last, loam_cloud_out* full_end,
                  int* published) {
  (void)stamp;
  if (!x || !in || !published) return fail(LOAM_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(x->device));
  *published = 0;
  SrBuffers& fi = x->odin;
  const int R = x->R;
  if (in->sharp.count > (uint32_t)(kSharpPerRing * R) || in->flat.count > (uint32_t)(kFlatPerRing * R) ||
      in->less_sharp.count > (uint32_t)(kLessSharpPerRing * R))
    return fail(LOAM_E_CAPACITY, "feature cloud larger than scan registration can produce");
  if (in->full.count > (uint32_t)x->cap) return fail(LOAM_E_CAPACITY, "input feature cloud exceeds capacity");
  if (in->full.count > 0 && in->full.pts == nullptr) return fail(LOAM_E_INVAL, "feature cloud pts is null");
  int rc = 0;
  x->pin.reset();
  HIP_TRY(x->pin.reserve((size_t)in->sharp.count + in->less_sharp.count + in->flat.count + in->less_flat.count +
                             in->full.count, x->st));
  // only k_od_end reads the full cloud: after the first frame, with a second stream, it is staged
  // while the L-M kernels run (late_full below)
  const bool late = x->od_inited && x->st2 != nullptr && in->full.count > 0;
  if ((rc = upload_cloud(x->st, x->pin, in->sharp, fi.sharp, kSharpPerRing * R)) ||
      (rc = upload_cloud(x->st, x->pin, in->less_sharp, fi.lsharp, kLessSharpPerRing * R)) ||
      (rc = upload_cloud(x->st, x->pin, in->flat, fi.flat, kFlatPerRing * R)) ||
      (rc = upload_cloud(x->st, x->pin, in->less_flat, fi.lflat, x->cap)) ||
      (!late && (rc = upload_cloud(x->st, x->pin, in->full, fi.full, x->cap))))
    return rc;
  int cnt[5] = {(int)in->sharp.count, (int)in->less_sharp.count, (int)in->flat.count,
                (int)in->less_flat.count, (int)in->full.count};
  {
    Xfer xp;
    xp.put(fi.cnt, cnt, 4 * sizeof(int));
    xp.put(fi.n_full, &cnt[4], sizeof(int));
    HIP_TRY(xfer_launch(xp, x->st));
    HIP_TRY(hipGetLastError());
  }
  return od_frame(x, feat_view(fi, 0, 1), cnt, in->imu_trans, late ? &in->full : nullptr, sum_out, corner_last,
                  surf_last, full_end, published, nullptr);
}
}  // extern "C"

namespace {
int od_frame(loam_ctx* x, const FeatView& fv, const int* cnt, const float* imu_in, const loam_cloud_out* late_full,
             loam_pose6* sum_out, loam_cloud_out* corner_last, loam_cloud_out* surf_last, loam_cloud_out* full_end,
             int* published, int* nl3, bool defer, bool sr_pending) {
  *published = 0;
  OdBuffers& o = x->od1;
  SrBuffers& fi = x->odin;
  int* mi = (int*)x->meta;  // [8..19] imu_trans, [24..] downloads below
  std::memcpy(mi + 8, imu_in, 12 * sizeof(float));
  const bool late = late_full != nullptr;
  std::memset(&x->stats, 0, sizeof(x->stats));
  // imuTransHandler (:330-351): this sweep's /imu_trans, in the state order load_imu reads
  {
    Xfer xp;
    xp.put(o.state + kOdImu, mi + 8, 12 * sizeof(float));
    HIP_TRY(xfer_launch(xp, x->st));
  }
  HIP_TRY(od_wait_hashes(o, x->st));  // (the previous frame's hash build, when deferred)
  if (!x->od_inited) {  // src/laserOdometry.cpp:427-456: Last = raw lessSharp / lessFlat, no L-M
    // :451-452 transformSum[0] += imuPitchStart; transformSum[2] += imuRollStart (from zero)
    const float sum0[3] = {0.0f + imu_in[0], 0.0f, 0.0f + imu_in[2]};
    HIP_TRY(hipMemcpyAsync(o.state + kOdSum, sum0, sizeof(sum0), hipMemcpyHostToDevice, x->st));
    x->od_sum[0] = sum0[0];
    x->od_sum[2] = sum0[2];
    hipLaunchKernelGGL(k_od_end, dim3(16, 1), dim3(256), 0, x->st, o, fv, 0, 0, 0);
    od_build_hashes(o, 0, x->st);
    HIP_TRY(hipGetLastError());
    x->od_last = 0;
    x->od_inited = true;
    int* nl = mi + 24;
    HIP_TRY(hipMemcpyAsync(nl, o.nlast, 2 * sizeof(int), hipMemcpyDeviceToHost, x->st));
    HIP_TRY(hipStreamSynchronize(x->st));
    *published = LOAM_PUB_CLOUDS;
    if (nl3) { nl3[0] = nl[0]; nl3[1] = nl[1]; nl3[2] = 0; }
    x->pin.reset();
    int e = copy_out(x->st, x->pin, o.lastC, nl[0], corner_last) | copy_out(x->st, x->pin, o.lastS, nl[1], surf_last);
    HIP_TRY(hipStreamSynchronize(x->st));
    x->pin.finish();
    return e ? LOAM_E_CAPACITY : LOAM_OK;
  }
  const int cur = x->od_last, nxt = 1 - cur;
  HIP_TRY(hipEventRecord(x->ev[0], x->st));
  // the pose accumulation (:830-856) runs on the host after the download: one scalar chain of
  // double trig, which a one-thread kernel took ~16 us for (the batch path keeps it on the device)
  // sr_pending: k_od_begin keeps a copy of the state to undo this frame with (the third state slot,
  // unused by the one-problem context)
  OdBuffers ob = o;
  const bool graph = x->tune.od_graph && defer;  // (the chain: fv is the context's own sr1)
  if (sr_pending || graph) {  // (a graph bakes the copy in: every replayed frame keeps it)
    ob.bk_state = o.state_set[2];
    ob.bk_istate = o.istate_set[2];
  }
  if (graph) {
    if (!x->od_graph_exec[cur]) {
      HIP_TRY(hipStreamBeginCapture(x->st, hipStreamCaptureModeThreadLocal));
      od_solve(ob, fv, cur, x->st, nullptr, /*device_fini=*/false);
      hipGraph_t g = nullptr;
      const hipError_t ce = hipGetLastError(), ee = hipStreamEndCapture(x->st, &g);
      if (ce != hipSuccess || ee != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        return fail(LOAM_E_HIP, std::string("odometry graph capture: ") + hipGetErrorString(ce != hipSuccess ? ce : ee));
      }
      x->od_graph[cur] = g;
      HIP_TRY(hipGraphInstantiate(&x->od_graph_exec[cur], g, nullptr, nullptr, 0));
    }
    HIP_TRY(hipGraphLaunch(x->od_graph_exec[cur], x->st));
  } else {
    od_solve(ob, fv, cur, x->st, nullptr, /*device_fini=*/false);
  }
  if (late) {  // late_full: host copy + DMA on the second stream, overlapping the L-M above
    HIP_TRY(x->pin.up(x->st2, fi.full, late_full->pts, (size_t)late_full->count));
    HIP_TRY(hipEventRecord(x->join, x->st2));
    HIP_TRY(hipStreamWaitEvent(x->st, x->join, 0));
  }
  const int frame_count0 = x->od_frame_count;
  x->od_frame_count++;
  const bool pub = x->od_frame_count >= (int)x->cfg.skip_frame_num + 1;
  hipLaunchKernelGGL(k_od_end, dim3(64, 1), dim3(256), 0, x->st, o, fv, nxt, 2, pub ? 1 : 0);  // one sweep: a wider grid
  // the new Last clouds' hash tables are read by the next frame's association only: with
  // stream_defer they are built on the second stream while this frame's results go out (and the
  // mapping runs)
  if (defer && x->tune.stream_defer && x->st2) HIP_TRY(od_build_hashes_deferred(o, nxt, x->st, x->st2));
  else od_build_hashes(o, nxt, x->st);
  HIP_TRY(hipEventRecord(x->ev[1], x->st));
  HIP_TRY(hipGetLastError());
  x->od_last = nxt;
  // state (kOdStateFloats), istate (kOdStateInts), nlast (4: problem 0's buffers 0 and 1, the two the
  // streaming path alternates), nfullEnd (2) into the mapped host
  // block in one launch, then copied out (the host edits st / ist below)
  static_assert(kXferOd + 4 * (kOdStateFloats + kOdStateInts + 6) <= kXferMp, "odometry transfer region");
  {
    Xfer xg;
    char* d = x->xb.d + kXferOd;
    xg.get(d, o.state, kOdStateFloats * sizeof(float));
    xg.get(d + 4 * kOdStateFloats, o.istate, kOdStateInts * sizeof(int));
    xg.get(d + 4 * (kOdStateFloats + kOdStateInts), o.nlast, 4 * sizeof(int));
    xg.get(d + 4 * (kOdStateFloats + kOdStateInts + 4), o.nfullEnd, 2 * sizeof(int));
    HIP_TRY(xfer_launch(xg, x->st));
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(x->st));
  int cnt_l[5];
  if (sr_pending) {  // the scan registration's result is known now
    const int src = sr_collect(x, cnt_l);
    cnt = cnt_l;
    if (src) {  // undo this frame: the state from k_od_begin's copy, the host counters (Last[nxt] unused)
      HIP_TRY(hipMemcpyAsync(o.state, o.state_set[2], kOdStateFloats * sizeof(float), hipMemcpyDeviceToDevice, x->st));
      HIP_TRY(hipMemcpyAsync(o.istate, o.istate_set[2], kOdStateInts * sizeof(int), hipMemcpyDeviceToDevice, x->st));
      HIP_TRY(hipStreamSynchronize(x->st));
      x->od_last = cur;
      x->od_frame_count = frame_count0;
      return src;
    }
  }
  float* st = (float*)(mi + 32);                  // kOdStateFloats
  int* ist = mi + 32 + kOdStateFloats;             // kOdStateInts
  int* nl = ist + kOdStateInts;                    // 4
  int* nfe = nl + 4;                               // 2
  std::memcpy(st, x->xb.h + kXferOd, 4 * (kOdStateFloats + kOdStateInts + 6));
  if (ist[kIsErr]) return fail(LOAM_E_CAPACITY, "odometry capacity exceeded");
  {  // :830-856 (k_od_fini's body, host side): transformSum from this frame's transform
    const float* q = imu_in;
    loampose::Imu m;
    m.pitchStart = q[0]; m.yawStart = q[1]; m.rollStart = q[2];
    m.pitchLast = q[3]; m.yawLast = q[4]; m.rollLast = q[5];
    m.shiftX = q[6]; m.shiftY = q[7]; m.shiftZ = q[8];
    m.veloX = q[9]; m.veloY = q[10]; m.veloZ = q[11];
    loampose::accumulate_pose(st, m, x->od_sum);
    ist[kIsQueries] = ist[kIsAssoc] * (cnt[0] + cnt[2]);
    // keep the device copy of transformSum current (it is seeded only on the init frame): the
    // host result goes back in k_xfer's arguments, ordered before the next frame's kernels
    Xfer xp;
    xp.put(o.state + kOdSum, x->od_sum, sizeof(loam_pose6));
    HIP_TRY(xfer_launch(xp, x->st));
    HIP_TRY(hipGetLastError());
  }
  if (sum_out) std::memcpy(sum_out, x->od_sum, sizeof(loam_pose6));
  *published = LOAM_PUB_POSE;
  int e = 0;
  if (pub) {
    x->od_frame_count = 0;
    *published |= LOAM_PUB_CLOUDS | LOAM_PUB_FULL;
    if (nl3) { nl3[0] = nl[nxt * 2 + 0]; nl3[1] = nl[nxt * 2 + 1]; nl3[2] = nfe[nxt]; }
    x->pin.reset();
    e |= copy_out(x->st, x->pin, o.lastC + (size_t)nxt * o.P * o.capC, nl[nxt * 2 + 0], corner_last);
    e |= copy_out(x->st, x->pin, o.lastS + (size_t)nxt * o.P * o.capS, nl[nxt * 2 + 1], surf_last);
    e |= copy_out(x->st, x->pin, o.fullEnd + (size_t)nxt * o.P * o.capS, nfe[nxt], full_end);
    HIP_TRY(hipStreamSynchronize(x->st));
    x->pin.finish();
  }
  float ms = 0;
  (void)hipEventElapsedTime(&ms, x->ev[0], x->ev[1]);
  x->stats.ms_od = ms;
  x->stats.od_iters = ist[kIsIters];
  x->stats.od_assoc_rounds = ist[kIsAssoc];
  x->stats.od_rows_sum = (uint64_t)ist[kIsRows];
  x->stats.od_queries = ist[kIsQueries];
  x->stats.od_degenerate_steps = (uint64_t)ist[kIsDegSteps];
  x->stats.od_nan_skips = (uint64_t)ist[kIsNanSkips];
  x->stats.od_assoc_gathered = (uint64_t)(uint32_t)ist[kIsGathered];
  x->stats.od_assoc_boxes = (uint64_t)(uint32_t)ist[kIsBoxes];
  {
    const uint64_t nq = ist[kIsAssoc] ? (uint64_t)(ist[kIsQueries] / ist[kIsAssoc]) : 0, it = (uint64_t)ist[kIsIters];
    x->stats.od_query_iters = nq * it;
    x->stats.od_row_evals = nq * it * (it + 1) / 2;
  }
  x->stats.od_corner_last = nl[cur * 2 + 0];
  x->stats.od_surf_last = nl[cur * 2 + 1];
  x->stats.od_assoc_points = (uint64_t)ist[kIsAssoc] * (nl[cur * 2 + 0] + nl[cur * 2 + 1]);
  count_bytes(x->stats);
  return e ? LOAM_E_CAPACITY : LOAM_OK;
}
}  // namespace

extern "C" {

// ------------------------------------------------------------------ laserMapping
int loam_mapping(loam_ctx* x, double stamp, const loam_pose6* odom_sum, const loam_cloud_out* corner_last,
                 const loam_cloud_out* surf_last, const loam_cloud_out* full_end, loam_pose6* aft,
                 loam_pose6* bef, loam_cloud_out* registered) {
  if (!x || !odom_sum || !corner_last || !surf_last || !full_end || !aft || !bef)
    return fail(LOAM_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(x->device));
  // transformUpdate's IMU blend (:199-226): roll / pitch at the odometry stamp + scanPeriod
  float rp[2];
  int front = 0;
  const bool have_imu = loamimu::mp_lookup(x->mp_imu, stamp, rp[0], rp[1], front);
  bool updated = false;
  const int rc = mp_stream_frame(x->mp1, x->st, *odom_sum, *corner_last, *surf_last, *full_end, aft, bef,
                                 registered, &x->stats, g_err, x->pin, x->io(), have_imu ? rp : nullptr, &updated,
                                 x->st2, x->join);
  if (have_imu && updated) x->mp_imu.front = front;  // the pointer walk happens inside transformUpdate
  x->surround_due = false;
  if (rc == LOAM_OK && ++x->map_frame_count >= 5) {  // :1038-1040
    x->map_frame_count = 0;
    x->surround_due = true;
  }
  return rc;
}

// ------------------------------------------------------------------ device-resident node chain
// scanRegistration -> laserOdometry -> laserMapping on one sweep with the intermediate topics left
// in device memory: odometry reads scanRegistration's buffers (sr1) in place and mapping reads
// odometry's published CornerLast / SurfLast / full-end buffers in place.  The arithmetic is the
// three node calls' own (the same kernels on the same values); only the host round trips of the
// intermediate clouds are gone, as in an intra-process (nodelet) deployment.
int loam_chain_sweep(loam_ctx* x, double stamp, loam_cloud_in raw, loam_chain_out* out) {
  if (!x || !out) return fail(LOAM_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(x->device));
  out->published = 0;
  out->mapped = 0;
  int cnt5[5];
  float imu12[12];
  // (stream_defer, after the odometry's first frame: the odometry is enqueued behind the scan
  // registration without a host round trip; sr_frame's pending mode)
  bool sr_pending = false;
  int rc = sr_frame(x, stamp, raw, nullptr, cnt5, imu12, x->od_inited && x->tune.stream_defer ? &sr_pending : nullptr);
  if (rc) return rc;
  int nl3[3] = {0, 0, 0};
  rc = od_frame(x, feat_view(x->sr1, 0, 1), cnt5, imu12, nullptr, &out->od_sum, nullptr, nullptr, nullptr,
                &out->published, nl3, /*defer=*/true, sr_pending);
  if (rc) return rc;
  if (out->published != (LOAM_PUB_POSE | LOAM_PUB_CLOUDS | LOAM_PUB_FULL)) return LOAM_OK;
  const OdBuffers& o = x->od1;
  const int nxt = x->od_last;  // od_frame swapped: the published Last is the current one
  MpInput in;
  in.corner = o.lastC + (size_t)nxt * o.P * o.capC;
  in.surf = o.lastS + (size_t)nxt * o.P * o.capS;
  in.full = o.fullEnd + (size_t)nxt * o.P * o.capS;
  in.corner_stride = o.capC; in.surf_stride = o.capS; in.full_stride = o.capS;
  in.ncorner = o.nlast + nxt * 2; in.nsurf = o.nlast + nxt * 2 + 1; in.nfull = o.nfullEnd + nxt;
  in.ncorner_stride = in.nsurf_stride = 2 * kOdBufs; in.nfull_stride = kOdBufs;
  in.pose = nullptr; in.pose_stride = 6;
  float rp[2];
  int front = 0;
  const bool have_imu = loamimu::mp_lookup(x->mp_imu, stamp, rp[0], rp[1], front);
  bool updated = false;
  loam_cloud_out* reg = out->registered.capacity ? &out->registered : nullptr;
  if (!reg) out->registered.count = 0;
  rc = mp_stream_frame_dev(x->mp1, x->st, out->od_sum, in, nl3, &out->aft, &out->bef, reg, &x->stats, g_err,
                           x->pin, x->io(), have_imu ? rp : nullptr, &updated, x->tune.stream_defer ? x->st2 : nullptr);
  if (have_imu && updated) x->mp_imu.front = front;
  x->surround_due = false;
  if (rc == LOAM_OK && ++x->map_frame_count >= 5) {  // :1038-1040
    x->map_frame_count = 0;
    x->surround_due = true;
  }
  if (rc == LOAM_OK) out->mapped = 1;
  return rc;
}

int loam_mapping_surround(loam_ctx* x, loam_cloud_out* out, int* published) {
  if (!x || !out || !published) return fail(LOAM_E_INVAL, "null argument");
  *published = 0;
  if (!x->surround_due) {
    out->count = 0;
    return LOAM_OK;
  }
  if (out->capacity && !out->pts) return fail(LOAM_E_INVAL, "surround cloud pts is null");
  HIP_TRY(hipSetDevice(x->device));
  const int rc = mp_stream_surround(x->mp1, x->st, out, g_err);
  if (rc == LOAM_OK) *published = 1;
  return rc;
}

// ------------------------------------------------------------------ IMU
int loam_imu(loam_ctx* x, double stamp, const double* quat_xyzw, const double* lin_acc_xyz) {
  if (!x || !quat_xyzw || !lin_acc_xyz) return fail(LOAM_E_INVAL, "null argument");
  if (!(stamp >= x->imu_last_stamp)) return fail(LOAM_E_INVAL, "IMU stamps must be non-decreasing");
  x->imu_last_stamp = stamp;
  double roll, pitch, yaw;
  loampose::rpy_from_quat(quat_xyzw, roll, pitch, yaw);  // tf::Matrix3x3(q).getRPY
  loamimu::sr_push(*x->sr_imu, stamp, roll, pitch, yaw, lin_acc_xyz);  // scanRegistration.cpp:638-660
  loamimu::mp_push(x->mp_imu, stamp, roll, pitch);                     // laserMapping.cpp:323-335
  return LOAM_OK;
}

// ------------------------------------------------------------------ transformMaintenance
int loam_maintenance(const loam_pose6* odom_sum, const loam_pose6* bef, const loam_pose6* aft,
                     loam_pose6* integrated) {
  if (!odom_sum || !bef || !aft || !integrated) return fail(LOAM_E_INVAL, "null argument");
  // src/transformMaintenance.cpp:147-203: Sum and Aft arrive as quaternion messages, Bef through
  // the twist fields; then transformAssociateToMap (:60-145).  Scalar host algebra, no kernel.
  float S[6], A[6], B[6], incre[6] = {0, 0, 0, 0, 0, 0}, T[6];
  loampose::pose_through_msg((const float*)odom_sum, S);
  loampose::pose_through_msg((const float*)aft, A);
  std::memcpy(B, bef, sizeof(B));
  loampose::associate_to_map(S, B, A, incre, T);
  std::memcpy(integrated, T, sizeof(T));
  return LOAM_OK;
}

// ------------------------------------------------------------------ batch (config 4)
int loam_batch_upload(loam_ctx* x, uint32_t n, const loam_cloud_in* prev, const loam_cloud_in* cur) {
  if (!x || !prev || !cur || n == 0) return fail(LOAM_E_INVAL, "bad batch arguments");
  HIP_TRY(hipSetDevice(x->device));
  for (uint32_t i = 0; i < n; ++i) {
    int rc = check_cloud_in(prev[i], x->cap);
    if (!rc) rc = check_cloud_in(cur[i], x->cap);
    if (rc) return rc;
  }
  // (a step ahead may still read the raw sweeps or write its buffer set)
  HIP_TRY(hipStreamSynchronize(x->st));
  if (x->st2) HIP_TRY(hipStreamSynchronize(x->st2));
  if (x->st3) HIP_TRY(hipStreamSynchronize(x->st3));
  if (x->st4) HIP_TRY(hipStreamSynchronize(x->st4));
  x->reset_ahead();
  x->fed = false;
  if ((int)n != x->P) {
    if (x->st2) HIP_TRY(hipStreamSynchronize(x->st2));
    x->drop_graph();  // (its kernels' arguments name the old buffers)
    x->free_feed();   // (sized for the old batch)
    sr_free(x->srb);
    sr_free(x->srb2);
    sr_free(x->srb3);
    od_free(x->odb);
    mp_free(x->mpb);
    mp_free(x->mpb2);
    x->P = 0;  // no batch until every buffer of the new size exists
    // (the second SR / mapping sets only when a mode that alternates them runs: ensure_second_sets)
    hipError_t he = sr_alloc(x->srb, 2 * (int)n, x->cap, x->R);
    if (he == hipSuccess) he = od_alloc(x->odb, (int)n, x->R, x->cap, (int)x->cfg.od_max_iter);
    if (he == hipSuccess)
      he = mp_alloc(x->mpb, (int)n, x->R, x->cap, mp_batch_map_capacity(x->cap), (int)x->cfg.mp_max_iter);
    if (he != hipSuccess) {
      sr_free(x->srb);
      sr_free(x->srb2);
      sr_free(x->srb3);
      od_free(x->odb);
      mp_free(x->mpb);
      mp_free(x->mpb2);
      return fail(LOAM_E_NOMEM, std::string("batch allocation failed: ") + hipGetErrorString(he));
    }
    x->P = (int)n;
  }
  x->odb.tune = x->tune;
  x->mpb.tune = x->mpb2.tune = x->tune;
  std::vector<float4> h((size_t)x->cap);
  std::vector<int> counts(2 * n);
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 2; ++k) {
      const loam_cloud_in& c = k == 0 ? prev[i] : cur[i];
      pack(c, h.data(), 0, c.count);
      counts[2 * i + k] = (int)c.count;
      HIP_TRY(hipMemcpy(x->srb.raw + (size_t)(2 * i + k) * x->cap, h.data(), (size_t)c.count * sizeof(float4),
                        hipMemcpyHostToDevice));
    }
  HIP_TRY(hipMemcpy(x->srb.raw_n, counts.data(), counts.size() * sizeof(int), hipMemcpyHostToDevice));
  for (SrBuffers* o : {&x->srb2, &x->srb3})
    if (o->S) {  // the other sets' raw sweeps (tune.sr_ahead / step_pipe)
      HIP_TRY(hipMemcpy(o->raw, x->srb.raw, (size_t)2 * n * x->cap * sizeof(float4), hipMemcpyDeviceToDevice));
      HIP_TRY(hipMemcpy(o->raw_n, x->srb.raw_n, counts.size() * sizeof(int), hipMemcpyDeviceToDevice));
    }
  return LOAM_OK;
}

namespace {
// sweeps [s0, s1) of a batch (sweep 2i = prev[i], 2i + 1 = cur[i]) packed back to back (sweep s at off[s]) into dst, on up to eight threads
void pack_tight(const loam_cloud_in* prev, const loam_cloud_in* cur, size_t s0, size_t s1, const int* off, float4* dst) {
  auto run = [&](size_t a, size_t b) {
    for (size_t s = a; s < b; ++s) {
      const loam_cloud_in& c = (s & 1) ? cur[s / 2] : prev[s / 2];
      pack(c, dst + off[s], 0, c.count);
    }
  };
  const size_t S = s1 - s0;
  const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  const size_t nt = S >= 64 ? hw : 1;
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(run, s0 + S * t / nt, s0 + S * (t + 1) / nt);
  run(s0, s0 + S / nt);
  for (auto& t : th) t.join();
}

// The second scan-registration set and the second mapping set, which only the modes that alternate
// the sets between steps use (tune.sr_ahead, tune.step_pipe): allocated on the first step that
// needs them, the uploaded raw sweeps copied from the first set.  The sets of the batch are then
// kept until an upload of another size.
// the SR sets the step pipeline rotates (tune.pipe_sr_sets when pipelined, else 2)
int pipe_slots(const loam_ctx* x, bool pipe) { return pipe ? x->tune.pipe_sr_sets : 2; }

int ensure_second_sets(loam_ctx* x, int slots) {
  const int P = x->P;
  if (slots > 2 && !x->srb3.S) {  // the third SR set (tune.pipe_sr_sets = 3)
    const hipError_t he = sr_alloc(x->srb3, 2 * P, x->cap, x->R);
    if (he != hipSuccess) {
      sr_free(x->srb3);
      return fail(LOAM_E_NOMEM, std::string("third batch set allocation failed: ") + hipGetErrorString(he));
    }
    HIP_TRY(hipMemcpy(x->srb3.raw, x->srb.raw, (size_t)2 * P * x->cap * sizeof(float4), hipMemcpyDeviceToDevice));
    HIP_TRY(hipMemcpy(x->srb3.raw_n, x->srb.raw_n, (size_t)2 * P * sizeof(int), hipMemcpyDeviceToDevice));
  }
  if (x->srb2.S) return LOAM_OK;
  hipError_t he = sr_alloc(x->srb2, 2 * P, x->cap, x->R);
  if (he == hipSuccess)
    he = mp_alloc(x->mpb2, P, x->R, x->cap, mp_batch_map_capacity(x->cap), (int)x->cfg.mp_max_iter);
  if (he != hipSuccess) {
    sr_free(x->srb2);
    sr_free(x->srb3);
    mp_free(x->mpb2);
    return fail(LOAM_E_NOMEM, std::string("second batch set allocation failed: ") + hipGetErrorString(he));
  }
  x->mpb2.tune = x->tune;
  // (the raw sweeps are only read by the kernels, so the first set's may be copied while steps run)
  HIP_TRY(hipMemcpy(x->srb2.raw, x->srb.raw, (size_t)2 * P * x->cap * sizeof(float4), hipMemcpyDeviceToDevice));
  HIP_TRY(hipMemcpy(x->srb2.raw_n, x->srb.raw_n, (size_t)2 * P * sizeof(int), hipMemcpyDeviceToDevice));
  return LOAM_OK;
}
}  // namespace

namespace {
// one batch step's device work on x->st (+ x->st2 for mapping frame 1); timing events only when
// `events` (a captured graph records none: its stage times are not split)
hipError_t batch_enqueue(loam_ctx* x, Prof* pf, bool events) {
  const int P = x->P;
  OdBuffers& o = x->odb;
  hipError_t e = hipSuccess;
  auto T = [&](hipError_t r) { if (e == hipSuccess) e = r; };
  // scan registration of this step: already enqueued one step ahead (st3), or here
  const int idx = x->sr_idx;
  SrBuffers& sb = x->srbuf(idx);
  const int ls = x->od_s, le = x->od_e;  // (Last buffers: the seed's, TransformToEnd's)
  x->od_s_last = ls;
  if (events) T(hipEventRecord(x->ev[0], x->st));
  x->prof.begin(x->st);
  if (x->b_used) {  // pipelined steps' mappings may still run on st4 / st2 (batch_enqueue_pipe)
    for (int i = 0; i < 3; ++i)
      if (x->mp_done_rec[i]) T(hipStreamWaitEvent(x->st, x->mp_done[i], 0));
    x->b_used = false;
  }
  if (x->sr_ready) {
    T(hipStreamWaitEvent(x->st, x->sr_done, 0));
    x->sr_ready = false;
  } else {
    sr_launch(sb, sr_params(x), x->st, pf);
  }
  if (events) T(hipEventRecord(x->ev[1], x->st));
  o.istate = o.istate_set[idx];  // (this step's; the kernels take the buffers by value)
  o.state = o.state_set[idx];
  T(hipMemsetAsync(o.state, 0, (size_t)P * kOdStateFloats * sizeof(float), x->st));
  const FeatView fprev = feat_view(sb, 0, 2), fcur = feat_view(sb, 1, 2);
  const bool ahead = x->st3 && x->tune.sr_ahead > 0 && P >= x->tune.sr_ahead && events && !pf;
  const int ahead_at = x->tune.sr_ahead_at >= 0 ? x->tune.sr_ahead_at : (P <= 256 ? 2 : 1);
  auto ahead_point = [&](int at) {
    if (ahead && ahead_at == at) T(hipEventRecord(x->ahead_at, x->st));
  };
  ahead_point(0);
  // odometry seeded from prev as a solved zero-increment frame, then one loop body on cur
  // (the full clouds' TransformToEnd happens in mapping's registration kernel, mp_batch_frame*)
  if (x->seed_ready) {  // enqueued one step ahead (st3, seed_done)
    T(hipStreamWaitEvent(x->st, x->seed_done, 0));
    x->seed_ready = false;
  } else {
    T(hipMemsetAsync(o.istate, 0, (size_t)P * kOdStateInts * sizeof(int), x->st));
    hipLaunchKernelGGL(k_od_end, dim3(kOdEndWg, P), dim3(256), 0, x->st, o, fprev, ls, 1, 0);
    x->prof.mark("k_od_end_seed");
    od_build_hashes(o, ls, x->st);
    x->prof.mark("k_hash_build_last");
  }
  ahead_point(1);
  // mapping frame 1 (prev into an empty map at the origin) reads only the seeding's Last[s]: it runs on a second stream beside the odometry solve, whose L-M iterations are
  // chains of small latency-bound launches that leave most of the chip idle.  The profiling pass
  // keeps one stream so that its per-kernel event times stay attributable.
  const bool overlap = x->st2 && !pf;
  if (overlap) {
    T(hipEventRecord(x->fork, x->st));
    T(hipStreamWaitEvent(x->st2, x->fork, 0));
    mp_batch_frame1(x->mpbuf(idx), o, ls, fprev, x->st2, nullptr);
    T(hipEventRecord(x->join, x->st2));
  }
  // the pose accumulation (k_od_fini, one serial double-trig chain per problem) beside
  // TransformToEnd on the second stream: both only read the solved transform
  od_solve(o, fcur, ls, x->st, pf, /*device_fini=*/!overlap);
  if (overlap) {
    T(hipEventRecord(x->fork2, x->st));
    T(hipStreamWaitEvent(x->st2, x->fork2, 0));
    od_fini(o, fcur, x->st2);
    T(hipEventRecord(x->join2, x->st2));
  }
  hipLaunchKernelGGL(k_od_end, dim3(kOdEndWg, P), dim3(256), 0, x->st, o, fcur, le, 2, 0);
  x->prof.mark("k_od_end");
  if (overlap) T(hipStreamWaitEvent(x->st, x->join2, 0));
  if (events) T(hipEventRecord(x->ev[2], x->st));
  // mapping: (frame 1 unless overlapped) then cur with the odometry pose
  if (overlap) {
    T(hipStreamWaitEvent(x->st, x->join, 0));
  } else {
    mp_batch_frame1(x->mpbuf(idx), o, ls, fprev, x->st, pf);
  }
  ahead_point(2);
  if (ahead) T(hipEventRecord(x->seed_at, x->st));
  // (frame 1 is done: the second stream is free for frame 2's independent branches)
  SideStream side;
  side.st = x->st2;
  side.fork[0] = x->fork; side.join[0] = x->join; side.fork[1] = x->fork2; side.join[1] = x->join2;
  mp_batch_frame2(x->mpbuf(idx), o, le, fcur, x->st, pf, overlap ? &side : nullptr);
  x->mp_last = idx;
  if (events) T(hipEventRecord(x->ev[3], x->st));
  x->srb_last = idx;
  // the next step's scan registration into the other set, once the step that last read it is done
  // (not in a captured graph, whose replays would all reuse one set, nor in the profiling pass)
  if (ahead) {
    T(hipEventRecord(x->step_done[idx], x->st));
    x->step_done_rec[idx] = true;
    const int nx = idx == 0 ? 1 : 0;  // (two sets here; a slot 2 left by pipelined runs goes back to 0)
    if (x->step_done_rec[nx]) T(hipStreamWaitEvent(x->st3, x->step_done[nx], 0));
    T(hipStreamWaitEvent(x->st3, x->ahead_at, 0));
    sr_launch(x->srbuf(nx), sr_params(x), x->st3, nullptr);
    T(hipEventRecord(x->sr_done, x->st3));
    x->sr_ready = true;
    x->sr_idx = nx;
    // the next step's odometry seed: Last[s] / its hashes are free once this step's odometry is
    // done (the second mapping frame reads Last[e] and the state only); its counts go to the other
    // istate set, which the next step reads
    T(hipStreamWaitEvent(x->st3, x->seed_at, 0));
    OdBuffers on = o;
    on.istate = o.istate_set[nx];
    T(hipMemsetAsync(on.istate, 0, (size_t)P * kOdStateInts * sizeof(int), x->st3));
    hipLaunchKernelGGL(k_od_end, dim3(kOdEndWg, P), dim3(256), 0, x->st3, on, feat_view(x->srbuf(nx), 0, 2), ls, 1, 0);
    od_build_hashes(on, ls, x->st3);
    T(hipEventRecord(x->seed_done, x->st3));
    x->seed_ready = true;
  }
  T(hipGetLastError());
  return e;
}
// The scan registration of the step reading buffer set i and its odometry seed (Last[ls], its
// hashes, the counts in istate set i), on st3.  Waits: the set's previous step is done with it
// (mp_done[i]: its mapping, the last reader, after that step's odometry), and, when `free_last` is
// recorded, Last[ls]'s last reader: frame 2 of the step before the current one (the rotation of
// batch_enqueue_pipe leaves Last[ls] to no running step's odometry or frame 1).
// the event after which the seed of the step reading SR slot j may rewrite its Last buffer: frame 2
// of the step two before it (slot j - 2 of n) read that buffer last (its inputs_read), if recorded
hipEvent_t seed_free_last(const loam_ctx* x, int j, int n) {
  const int k = (j + n - 2) % n;
  return x->inputs_read_rec[k] ? x->inputs_read[k] : nullptr;
}
hipError_t enqueue_ahead(loam_ctx* x, int i, int ls, hipEvent_t free_last) {
  const int P = x->P;
  OdBuffers on = x->odb;
  hipError_t e = hipSuccess;
  auto T = [&](hipError_t r) { if (e == hipSuccess) e = r; };
  if (x->mp_done_rec[i]) T(hipStreamWaitEvent(x->st3, x->mp_done[i], 0));
  T(hipStreamWaitEvent(x->st3, x->a_start, 0));  // (whatever ran on st before this call)
  PT_BEGIN("sr", x->st3);
  sr_launch(x->srbuf(i), sr_params(x), x->st3, nullptr);
  PT_END("sr", x->st3);
  T(hipEventRecord(x->sr_done, x->st3));
  if (free_last) T(hipStreamWaitEvent(x->st3, free_last, 0));
  on.istate = on.istate_set[i];
  T(hipMemsetAsync(on.istate, 0, (size_t)P * kOdStateInts * sizeof(int), x->st3));
  hipLaunchKernelGGL(k_od_end, dim3(kOdEndWg, P), dim3(256), 0, x->st3, on, feat_view(x->srbuf(i), 0, 2), ls, 1, 0);
  od_build_hashes(on, ls, x->st3);
  T(hipEventRecord(x->seed_done, x->st3));
  x->sr_ready = x->seed_ready = true;
  return e;
}

// One batch step as a stage of a software pipeline over consecutive steps (tune.step_pipe):
//   st3  scan registration + odometry seed of step k + 1 (enqueue_ahead)
//   st   odometry of step k (L-M against Last[s], pose accumulation, TransformToEnd into Last[e])
//   st4 / st2  mapping of step k: frame 1 (reads Last[s]), frame 2 (reads Last[e], after the
//        odometry); with two mapping sets (tune.pipe_mp_sets = 2) the steps alternate st4 / st2
// so the odometry of step k + 1 runs beside the mapping of step k and the seed of step k + 2 beside
// both.  Buffers shared between steps: the SR set, the odometry state / istate sets and the mapping
// sets alternate; the three Last buffers rotate (s, e) -> (3 - s - e, s): step k + 1 seeds the one
// step k - 1's frame 2 read last (inputs_read of that parity), and step k + 1's TransformToEnd
// rewrites step k's Last[s] once frame 1 of step k has read it (mp1_read; the odometry of step k is
// ahead on st).  Every step does the same work as batch_enqueue's; loam_batch_sync waits for all
// four streams.
hipError_t batch_enqueue_pipe(loam_ctx* x) {
  const int P = x->P;
  OdBuffers& o = x->odb;
  hipError_t e = hipSuccess;
  auto T = [&](hipError_t r) { if (e == hipSuccess) e = r; };
  const int n = pipe_slots(x, true), idx = x->sr_idx, nx = (idx + 1) % n;
  const int ls = x->od_s, le = x->od_e, lf = kOdBufs - ls - le;
  static_assert(kOdBufs == 3, "the rotation takes three Last buffers");
  SrBuffers& sb = x->srbuf(idx);
  T(hipEventRecord(x->a_start, x->st));
  T(hipEventRecord(x->ev[0], x->st));
  // (not enqueued ahead: the first pipelined step, or a fed context's step without a feed, which
  // re-runs the set's resident sweeps; Last[ls]'s last reader as for the trailing call below)
  if (!x->sr_ready || !x->seed_ready) T(enqueue_ahead(x, idx, ls, seed_free_last(x, idx, n)));
  x->sr_ready = x->seed_ready = false;
  x->od_s_last = ls;
  const FeatView fprev = feat_view(sb, 0, 2), fcur = feat_view(sb, 1, 2);
  // odometry (st)
  o.istate = o.istate_set[idx];
  o.state = o.state_set[idx];
  T(hipStreamWaitEvent(x->st, x->sr_done, 0));
  T(hipStreamWaitEvent(x->st, x->seed_done, 0));
  T(hipEventRecord(x->ev[1], x->st));
  PT_BEGIN("od", x->st);
  T(hipMemsetAsync(o.state, 0, (size_t)P * kOdStateFloats * sizeof(float), x->st));
  od_solve(o, fcur, ls, x->st, nullptr, /*device_fini=*/true);
  // Last[le] was the previous step's Last[s]: its frame 1 has read it (its odometry is ahead on st);
  // before that, frame 2 of the step before read it, which the previous seed waited for
  if (x->b_used) T(hipStreamWaitEvent(x->st, x->mp1_read, 0));
  hipLaunchKernelGGL(k_od_end, dim3(kOdEndWg, P), dim3(256), 0, x->st, o, fcur, le, 2, 0);
  PT_END("od", x->st);
  T(hipEventRecord(x->od_done, x->st));
  T(hipEventRecord(x->ev[2], x->st));
  // mapping: frame 1 once the seed (and this call's earlier work on st) is there, frame 2 once the
  // odometry is.  tune.pipe_mp_sets = 2: the steps alternate between two mapping sets on st4 / st2,
  // so the next step's frame 1 runs beside this step's frame 2 (no side branches then); 1: one set
  // on st4, frame 2's independent branches on st2
  const bool two = x->tune.pipe_mp_sets == 2;
  const int m = x->pipe_k++ & 1;  // (the mapping sets alternate by step, whatever the SR slots)
  hipStream_t ms = two && m ? x->st2 : x->st4;
  MpBuffers& mb = two ? x->mpbuf(m) : x->mpb;
  T(hipStreamWaitEvent(ms, x->a_start, 0));
  T(hipStreamWaitEvent(ms, x->seed_done, 0));
  SideStream side1;  // (no branches: only the event once Last[ls] is read)
  side1.inputs_read = x->mp1_read;
  PT_BEGIN("mp1", ms);
  mp_batch_frame1(mb, o, ls, fprev, ms, nullptr, &side1);
  PT_END("mp1", ms);
  T(hipEventRecord(x->mp1_done, ms));
  T(hipStreamWaitEvent(ms, x->od_done, 0));
  PT_BEGIN("mp2", ms);
  SideStream side;
  side.st = two ? nullptr : x->st2;
  side.fork[0] = x->fork; side.join[0] = x->join; side.fork[1] = x->fork2; side.join[1] = x->join2;
  side.inputs_read = x->inputs_read[idx];
  mp_batch_frame2(mb, o, le, fcur, ms, nullptr, &side);
  PT_END("mp2", ms);
#ifdef LOAM_PIPE_TRACE
  ++g_pt.step;
#endif
  T(hipEventRecord(x->mp_done[idx], ms));
  x->mp_done_rec[idx] = true;
  x->b_used = true;
  x->mp_last = two ? m : 0;
  T(hipEventRecord(x->ev[3], ms));
  x->srb_last = idx;
  // the next step's scan registration + seed (st3) into Last[lf], which frame 2 of the previous
  // step (SR set nx) read last; a fed context's next loam_batch_feed enqueues them instead, after
  // copying its sweeps into set nx
  if (!x->fed) T(enqueue_ahead(x, nx, lf, seed_free_last(x, nx, n)));
  x->inputs_read_rec[idx] = true;
  x->od_s = lf;
  x->od_e = ls;
  x->sr_idx = nx;
  T(hipGetLastError());
  return e;
}
}  // namespace

int loam_batch_run(loam_ctx* x) {
  if (!x || x->P == 0) return fail(LOAM_E_INVAL, "no batch uploaded");
  HIP_TRY(hipSetDevice(x->device));
  Prof* pf = x->prof.on ? &x->prof : nullptr;
  const bool pipe = !pf && !x->tune.graph && x->st2 && x->st3 && x->st4 && x->tune.step_pipe > 0 && x->P >= x->tune.step_pipe;
  const bool ahead = !pf && !x->tune.graph && x->st3 && x->tune.sr_ahead > 0 && x->P >= x->tune.sr_ahead;
  if (pipe || ahead) {
    const int rc = ensure_second_sets(x, pipe_slots(x, pipe));
    if (rc) return rc;
  }
  if (pipe) {
    HIP_TRY(batch_enqueue_pipe(x));
    return LOAM_OK;
  }
  if (!x->tune.graph || pf) {
    HIP_TRY(batch_enqueue(x, pf, true));
    return LOAM_OK;
  }
  // graph replay: captured on the first call for this batch (the kernels' arguments are the
  // batch's buffers, which stay put until the next loam_batch_upload of another size)
  if (!x->graph_exec || x->graph_P != x->P) {
    x->drop_graph();
    HIP_TRY(hipStreamBeginCapture(x->st, hipStreamCaptureModeThreadLocal));
    const hipError_t ce = batch_enqueue(x, nullptr, false);
    hipGraph_t g = nullptr;
    const hipError_t ee = hipStreamEndCapture(x->st, &g);
    if (ce != hipSuccess || ee != hipSuccess) {
      if (g) (void)hipGraphDestroy(g);
      return fail(LOAM_E_HIP, std::string("batch graph capture: ") + hipGetErrorString(ce != hipSuccess ? ce : ee));
    }
    x->graph = g;
    HIP_TRY(hipGraphInstantiate(&x->graph_exec, g, nullptr, nullptr, 0));
    x->graph_P = x->P;
  }
  HIP_TRY(hipEventRecord(x->ev[0], x->st));
  HIP_TRY(hipEventRecord(x->ev[1], x->st));
  HIP_TRY(hipEventRecord(x->ev[2], x->st));
  HIP_TRY(hipGraphLaunch(x->graph_exec, x->st));
  HIP_TRY(hipEventRecord(x->ev[3], x->st));
  return LOAM_OK;
}

int loam_batch_feed(loam_ctx* x, uint32_t n, const loam_cloud_in* prev, const loam_cloud_in* cur) {
  if (!x || !prev || !cur || n == 0) return fail(LOAM_E_INVAL, "bad batch arguments");
  if (x->P == 0 || (int)n != x->P)
    return fail(LOAM_E_INVAL, "loam_batch_feed: n must equal the uploaded batch size (loam_batch_upload first)");
  HIP_TRY(hipSetDevice(x->device));
  for (uint32_t i = 0; i < n; ++i) {
    int rc = check_cloud_in(prev[i], x->cap);
    if (!rc) rc = check_cloud_in(cur[i], x->cap);
    if (rc) return rc;
  }
  const int P = x->P;
  const bool pipe = !x->prof.on && !x->tune.graph && x->st2 && x->st3 && x->st4 && x->tune.step_pipe > 0 &&
                    P >= x->tune.step_pipe;
  if (!pipe) {  // sequential steps: the next step's sweeps replace the resident ones (as an upload)
    return loam_batch_upload(x, n, prev, cur);
  }
  int rc = ensure_second_sets(x, pipe_slots(x, true));
  if (rc) return rc;
  const int i = x->sr_idx;  // the set the next step reads
  if (x->sr_ready || x->seed_ready) {
    // (enqueued ahead on the set's resident sweeps by a run before the context was fed: discarded,
    // the feed's scan registration rewrites the set)
    HIP_TRY(hipStreamSynchronize(x->st3));
    x->sr_ready = x->seed_ready = false;
  }
  const size_t per = (size_t)2 * P * x->cap;
  if (!x->feed_pin[i]) {
    HIP_TRY(hipHostMalloc((void**)&x->feed_pin[i], per * sizeof(float4), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&x->feed_n[i], (size_t)4 * P * sizeof(int), hipHostMallocDefault));
  }
  if (!x->feed_dev) {
    HIP_TRY(hipMalloc((void**)&x->feed_dev, per * sizeof(float4)));
    HIP_TRY(hipMalloc((void**)&x->feed_doff, (size_t)4 * P * sizeof(int)));
  }
  if (x->feed_rec[i]) HIP_TRY(hipEventSynchronize(x->feed_copied[i]));  // (the staging's last copy is out)
  SrBuffers& sb = x->srbuf(i);
  // behind the set's last reader (the step that used it: its mapping, after its scan registration)
  if (x->mp_done_rec[i]) HIP_TRY(hipStreamWaitEvent(x->st3, x->mp_done[i], 0));
  // the sweeps packed back to back in chunks, each chunk one copy into the device staging enqueued
  // before the next is packed (the host packing overlaps the DMA of the chunk before); then one
  // kernel puts every sweep at its stride in the set's raw array
  const size_t S = (size_t)2 * P;
  int* nn = x->feed_n[i];
  int* off = nn + S;
  {
    size_t run = 0;
    for (size_t s = 0; s < S; ++s) {
      const loam_cloud_in& c = (s & 1) ? cur[s / 2] : prev[s / 2];
      nn[s] = (int)c.count;
      off[s] = (int)run;
      run += c.count;
    }
  }
  constexpr size_t kFeedChunk = 128;  // sweeps
  for (size_t s0 = 0; s0 < S; s0 += kFeedChunk) {
    const size_t s1 = std::min(S, s0 + kFeedChunk);
    pack_tight(prev, cur, s0, s1, off, x->feed_pin[i]);
    const size_t a = (size_t)off[s0], b = (size_t)off[s1 - 1] + (size_t)nn[s1 - 1];
    if (b > a)
      HIP_TRY(hipMemcpyAsync(x->feed_dev + a, x->feed_pin[i] + a, (b - a) * sizeof(float4), hipMemcpyHostToDevice, x->st3));
  }
  HIP_TRY(hipMemcpyAsync(x->feed_doff, nn, 2 * S * sizeof(int), hipMemcpyHostToDevice, x->st3));
  HIP_TRY(sr_scatter_packed(x->feed_dev, x->feed_doff + S, x->feed_doff, sb.raw, x->cap, (int)S, x->st3));
  HIP_TRY(hipMemcpyAsync(sb.raw_n, x->feed_doff, S * sizeof(int), hipMemcpyDeviceToDevice, x->st3));
  HIP_TRY(hipEventRecord(x->feed_copied[i], x->st3));
  x->feed_rec[i] = true;
  HIP_TRY(enqueue_ahead(x, i, x->od_s, seed_free_last(x, i, pipe_slots(x, true))));
  x->fed = true;
  return LOAM_OK;
}

int loam_batch_sync(loam_ctx* x) {
  if (!x) return fail(LOAM_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(x->device));
  HIP_TRY(hipStreamSynchronize(x->st));
  // (a step's work includes its mapping on st4 and the scan registration it enqueued for the next
  // step on st3)
  if (x->st4) HIP_TRY(hipStreamSynchronize(x->st4));
  if (x->st2) HIP_TRY(hipStreamSynchronize(x->st2));
  if (x->st3) HIP_TRY(hipStreamSynchronize(x->st3));
  // launch errors of either mapping set (the step pipeline alternates them), reported by this call
  for (int i = 0; i < 2; ++i) HIP_TRY(x->mpbuf(i).take_error());
#ifdef LOAM_PIPE_TRACE
  g_pt.dump();
#endif
  return LOAM_OK;
}

int loam_batch_lm_info(loam_ctx* x, int32_t* od_iters, int32_t* mp_iters, loam_pose6* od_transform) {
  if (!x || x->P == 0) return fail(LOAM_E_INVAL, "no batch");
  HIP_TRY(hipSetDevice(x->device));
  const int P = x->P;
  for (hipStream_t s : {x->st, x->st2, x->st3, x->st4})
    if (s) HIP_TRY(hipStreamSynchronize(s));
  if (od_iters) {
    std::vector<int> ist((size_t)P * kOdStateInts);
    HIP_TRY(hipMemcpy(ist.data(), x->odb.istate, ist.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int i = 0; i < P; ++i) od_iters[i] = ist[(size_t)i * kOdStateInts + kIsIters];
  }
  if (od_transform) {  // (state floats 0..5: the L-M transform, kOdSum the accumulated pose)
    std::vector<float> st((size_t)P * kOdStateFloats);
    HIP_TRY(hipMemcpy(st.data(), x->odb.state, st.size() * sizeof(float), hipMemcpyDeviceToHost));
    for (int i = 0; i < P; ++i) std::memcpy(&od_transform[i], &st[(size_t)i * kOdStateFloats], sizeof(loam_pose6));
  }
  if (mp_iters) HIP_TRY(mp_batch_iters(x->mpbuf(x->mp_last), x->st, mp_iters));
  return LOAM_OK;
}

int loam_batch_download(loam_ctx* x, loam_pose6* od_sum, loam_pose6* aft, loam_stats* stats) {
  if (!x || x->P == 0) return fail(LOAM_E_INVAL, "no batch");
  HIP_TRY(hipSetDevice(x->device));
  const int P = x->P;
  HIP_TRY(hipStreamSynchronize(x->st));
  if (x->st4) HIP_TRY(hipStreamSynchronize(x->st4));
  if (x->st2) HIP_TRY(hipStreamSynchronize(x->st2));
  if (x->st3) HIP_TRY(hipStreamSynchronize(x->st3));  // (the work enqueued ahead rewrites Last[0] alike)
  std::vector<float> st((size_t)P * kOdStateFloats);
  std::vector<int> ist((size_t)P * kOdStateInts), srerr(2 * P), cnt(8 * P), nfull(2 * P), nl((size_t)kOdBufs * 2 * P);
  HIP_TRY(hipMemcpy(st.data(), x->odb.state, st.size() * sizeof(float), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(ist.data(), x->odb.istate, ist.size() * sizeof(int), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(srerr.data(), x->srbuf(x->srb_last).err, srerr.size() * sizeof(int), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(cnt.data(), x->srbuf(x->srb_last).cnt, cnt.size() * sizeof(int), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(nfull.data(), x->srbuf(x->srb_last).n_full, nfull.size() * sizeof(int), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(nl.data(), x->odb.nlast, nl.size() * sizeof(int), hipMemcpyDeviceToHost));
  for (int i = 0; i < 2 * P; ++i) {
    int rc = sr_errors(srerr[i]);
    if (rc) return rc;
  }
  if (od_sum)
    for (int i = 0; i < P; ++i) std::memcpy(&od_sum[i], &st[(size_t)i * kOdStateFloats + kOdSum], sizeof(loam_pose6));
  loam_stats s;
  std::memset(&s, 0, sizeof(s));
  // (a launch error recorded on the other mapping set during an earlier pipelined step fails this
  // call too, not a later unrelated one)
  HIP_TRY(x->mpbuf(1 - x->mp_last).take_error());
  int rc = mp_batch_download(x->mpbuf(x->mp_last), x->st, aft, &s, g_err);
  if (rc) return rc;
  for (int i = 0; i < 2 * P; ++i) {
    s.n_ring += nfull[i];
    s.n_sharp += cnt[4 * i]; s.n_less_sharp += cnt[4 * i + 1];
    s.n_flat += cnt[4 * i + 2]; s.n_less_flat += cnt[4 * i + 3];
  }
  int raw_n[2];
  (void)raw_n;
  std::vector<int> rn(2 * P);
  HIP_TRY(hipMemcpy(rn.data(), x->srbuf(x->srb_last).raw_n, rn.size() * sizeof(int), hipMemcpyDeviceToHost));
  for (int i = 0; i < 2 * P; ++i) s.n_raw += rn[i];
  const int ls = x->od_s_last;  // (the last step's Last[s]; every step reads the same counts)
  for (int i = 0; i < P; ++i) {
    const int* q = &ist[(size_t)i * kOdStateInts];
    if (q[kIsErr]) return fail(LOAM_E_CAPACITY, "odometry capacity exceeded");
    s.od_iters += q[kIsIters];
    s.od_assoc_rounds += q[kIsAssoc];
    s.od_rows_sum += (uint64_t)q[kIsRows];
    s.od_queries += q[kIsQueries];
    s.od_degenerate_steps += (uint64_t)q[kIsDegSteps];
    s.od_nan_skips += (uint64_t)q[kIsNanSkips];
    s.od_assoc_gathered += (uint64_t)(uint32_t)q[kIsGathered];
    s.od_assoc_boxes += (uint64_t)(uint32_t)q[kIsBoxes];
    const uint64_t nq = q[kIsAssoc] ? (uint64_t)(q[kIsQueries] / q[kIsAssoc]) : 0, it = (uint64_t)q[kIsIters];
    s.od_query_iters += nq * it;
    s.od_row_evals += nq * it * (it + 1) / 2;
    const int* n = &nl[((size_t)i * kOdBufs + ls) * 2];
    s.od_corner_last += n[0];
    s.od_surf_last += n[1];
    s.od_assoc_points += (uint64_t)q[kIsAssoc] * (n[0] + n[1]);
  }
  count_bytes(s);
  x->prof.collect();
  float ms_sr = 0, ms_od = 0, ms_mp = 0;
  (void)hipEventElapsedTime(&ms_sr, x->ev[0], x->ev[1]);
  (void)hipEventElapsedTime(&ms_od, x->ev[1], x->ev[2]);
  (void)hipEventElapsedTime(&ms_mp, x->ev[2], x->ev[3]);
  s.ms_sr = ms_sr;
  s.ms_od = ms_od;
  s.ms_mp = ms_mp;
  x->stats = s;
  if (stats) *stats = s;
  return LOAM_OK;
}

}  // extern "C"

namespace loam {
__global__ __launch_bounds__(256) void k_xfer(Xfer x) {
  for (int e = 0; e < x.n; ++e) {
    uint32_t* d = x.dst[e];
    const uint32_t* s = x.src[e];
    for (int w = threadIdx.x; w < x.words[e]; w += 256) d[w] = s ? s[w] : x.imm[x.imm_off[e] + w];
  }
}
hipError_t xfer_launch(const Xfer& x, hipStream_t st) {
  if (x.overflow) return hipErrorInvalidValue;
  if (x.n) hipLaunchKernelGGL(k_xfer, dim3(1), dim3(256), 0, st, x);
  return hipGetLastError();
}
}  // namespace loam
