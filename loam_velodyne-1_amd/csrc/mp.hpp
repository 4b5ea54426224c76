// Mapping device buffers and entry points (engine-internal).
#ifndef LOAM_MP_HPP
#define LOAM_MP_HPP

#include <hip/hip_runtime.h>

#include <functional>
#include <string>

#include "engine.hpp"
#include "xfer.hpp"
#include "od.hpp"

namespace loam {

// cube grid of src/laserMapping.cpp:64-70
constexpr int kCubeW = 21, kCubeH = 11, kCubeD = 21, kCubeNum = kCubeW * kCubeH * kCubeD;
constexpr int kMaxValid = 125;
constexpr int kMpFitGridMax = 256;  // k_mp_fit<true> workgroups per instance (partials per instance)
constexpr int kMpSmallGrid = 256;  // workgroups per instance of the small-batch L-M iteration (multiple of 8)

// per-instance float state: Sum | Incre | TobeMapped | Bef | Aft | matP[36] | pointOnYAxis[3]
constexpr int kMpSum = 0, kMpIncre = 6, kMpTobe = 12, kMpBef = 18, kMpAft = 24, kMpMatP = 30, kMpOnY = 66,
              kMpImuRP = 69, kMpStateFloats = 72;  // kMpImuRP: IMU (roll, pitch) for transformUpdate
enum { kMiCenW = 0, kMiCenH, kMiCenD, kMiDegen, kMiNValid, kMiIters, kMiRows, kMiStackC, kMiStackS, kMiFromC,
       kMiFromS, kMiErr, kMiLmRan, kMiValidPts, kMiStop, kMiFits, kMiImu, kMiCubeI, kMiCubeJ, kMiCubeK,
       kMiDegSteps,  // L-M updates of this frame projected by the iteration-0 degeneracy analysis
       kMiShifts,    // cube-grid slab shifts of this frame's recentring (the reference's passes)
       kMiNnCand,    // map points the 5-NN evaluated this frame (seeds included)
       kMiNnCells,   // hash bucket ranges the 5-NN read this frame
       kMpStateInts = 28 };
static_assert(kMiNnCells < kMpStateInts, "istate layout");

// one mapping frame's inputs for every instance (device pointers)
struct MpInput {
  const float4 *corner, *surf, *full;
  size_t corner_stride, surf_stride, full_stride;
  const int *ncorner, *nsurf, *nfull;
  int ncorner_stride, nsurf_stride, nfull_stride;
  const float* pose;   // transformSum of the odometry message (nullptr = zero pose)
  int pose_stride;
  // the batch path: `full` is the raw ring-sorted cloud, and k_mp_register applies odometry's
  // TransformToEnd itself (end_mode 1: zero transform, 2: the transform in end_state, OdBuffers
  // state layout), so the full cloud is neither written to nor read back from fullEnd
  const float* end_state = nullptr;
  int end_mode = 0;
};

// the voxel frame of a segment (PCL VoxelGrid's min_b and divb multipliers), for sub-segments that
// take their parent's (vg_run's big-segment split)
struct VgFrame {
  int m0, m1, m2, divx, divy, pad;
};

// segmented PCL VoxelGrid job (segment s: input in[begin[s] .. end[s]), output out[begin[s] ..))
struct VgJob {
  const float4* in;
  float4* out;
  const int* begin;
  const int* end;
  const float* leaf;     // per segment
  int* out_count;        // per segment
  uint32_t *keys, *keys_alt, *vals, *vals_alt;  // k_vg_big's global sort arrays (indexed like in)
  int nseg;
  int total;             // size of in / out / keys arrays
  // vg_run's cascade: lists[0] / lists[1] ([nseg] segment ids) and their lengths counts[0] / [1]
  // (device); a kernel processes every segment, or the ids of list / *list_n, and appends the
  // segments beyond its capacity to big / *big_n
  int* lists[2] = {nullptr, nullptr};
  int* counts = nullptr;   // [3]: the two lists' lengths, and the length of the caller's input list
  // set by the caller: counts[0] / counts[1] already zeroed by an earlier kernel on the stream
  bool zeroed = false;
  const int* list = nullptr;
  const int* list_n = nullptr;
  int* big = nullptr;
  int* big_n = nullptr;
  // incremental cube VoxelGrid (k_vg_merge): per segment the count of its leading points that are the
  // cube's previous VoxelGrid output, the candidate list, and the per-segment "done" flags the
  // cascade's first kernel skips
  const int* nold = nullptr;
  const int* mlist = nullptr;
  const int* mlist_n = nullptr;
  int* skip = nullptr;
  // per segment: the voxel frame to use instead of the segment's own bounding box (sub-segments of a
  // split parent); nullptr: every segment computes its own
  const VgFrame* frame = nullptr;
  int grid_max = 1 << 30;  // the first kernel's grid at most (the split's sub-job)
};

// vg_run's split of the segments beyond the LDS tiers (the HDL-64E surf stacks): each parent's
// points re-ordered stably into 16 buckets by the top bits of their voxel key (k_vg_split), the
// buckets VoxelGridded as sub-segments in the parent's frame by the LDS cascade, their outputs
// concatenated in bucket order (k_vg_join).  Sub-segment li * 16 + d; pts / out indexed like the
// job's input
struct VgSplit {
  float4* pts = nullptr;
  float4* out = nullptr;
  int *begin = nullptr, *end = nullptr, *out_count = nullptr;
  float* leaf = nullptr;
  VgFrame* frame = nullptr;
  int* lists[2] = {nullptr, nullptr};
  int* ilist = nullptr;   // the non-empty sub-segments (the cascade's input list)
  int* counts = nullptr;  // [3]: the cascade's two lists, ilist
  int npar = 0;           // parents it holds (list entries beyond go to k_vg_big)
};

struct MpBuffers {
  int P = 0, capC = 0, capS = 0, cap_stack = 0, map_cap = 0, max_iter = 10, tmax = 0;
  int pool_cur = 0;
  float* state = nullptr;     // [P][kMpStateFloats]
  int* istate = nullptr;      // [P][kMpStateInts]
  int* slots = nullptr;       // [2][P][kCubeNum][4] (offC, cntC, offS, cntS) per pool
  float4* pool = nullptr;     // [2][P][map_cap]
  int* valid = nullptr;       // [P][kMaxValid]
  int* vpre = nullptr;        // [P][kMaxValid + 1][2] FromMap prefix (corner, surf)
  // streaming inputs
  float4 *inC = nullptr, *inS = nullptr, *inF = nullptr;
  int* in_n = nullptr;        // [P][3]
  float* in_pose = nullptr;   // [P][6]
  // stacks
  float4* stack2 = nullptr;   // [P][cap_stack] corner at 0, surf at capC
  float4* stack = nullptr;    // [P][cap_stack] voxel-grid output (same layout)
  int* nstack = nullptr;      // [P][2]
  // FromMap + hashes
  float4* from = nullptr;     // [P][map_cap] corner then surf
  int *hC_start = nullptr, *hS_start = nullptr, *h_fill = nullptr, *hC_T = nullptr, *hS_T = nullptr;
  uint32_t *hC_rec = nullptr, *hS_rec = nullptr;  // [P][tmax] packed bucket ranges (HashJob::rec)
  float4 *hC_pts = nullptr, *hS_pts = nullptr;   // [P][map_cap]
  int* nfrom = nullptr;       // [P][2]
  // per-query L-M outputs of the current iteration
  int8_t* q_ok = nullptr;     // [P][cap_stack]
  float4* q_cf = nullptr;     // [P][cap_stack]
  int4* q_nn = nullptr;       // [P][cap_stack][2] this iteration's ordered 5-NN (i0..i3 | i4, d4 bits)
  float4* q_fit = nullptr;    // [P][cap_stack][4] MpFit: the 5-NN a line / plane was fitted to + the fit
                              // (k_mp_nnfit: the last iteration's 5-NN, distinct, fit-valid + the fit)
  // insertion / per-cube downsampling
  int* app_cnt = nullptr;     // [P][kCubeNum][2] appended points per cube
  int* citems = nullptr;      // [P][2 * kCubeNum] non-empty (kind, cube, valid index) of the new store
  int* nitems = nullptr;      // [P]
  int* app_off = nullptr;     // [P][kCubeNum][2]
  float4* app = nullptr;      // [P][cap_stack] stack points grouped by cube (map frame)
  float4* vin = nullptr;      // [P][map_cap] per-valid-cube DS input (old ++ appended)
  float4* vout = nullptr;     // [P][map_cap]
  int *vseg_b = nullptr, *vseg_e = nullptr, *vseg_cnt = nullptr;  // [P][2*kMaxValid]
  float* vseg_leaf = nullptr;
  int *sseg_b = nullptr, *sseg_e = nullptr, *sseg_cnt = nullptr;  // [P][2] stack segments
  float* sseg_leaf = nullptr;
  uint32_t *vg_k = nullptr, *vg_k2 = nullptr, *vg_v = nullptr, *vg_v2 = nullptr;
  int *vg_l0 = nullptr, *vg_l1 = nullptr;  // [P][2][kMaxValid] vg_run's segment lists
  int* vg_lin = nullptr;                   // [P][2][kMaxValid] the non-empty cube segments (k_mp_vseg)
  int* vg_cnt = nullptr;                   // [4] the lists' lengths (vg_l0, vg_l1, vg_lin, vg_mlist)
  int* vg_mlist = nullptr;                 // [P][2][kMaxValid] cube segments k_vg_merge may take
  int* vseg_nold = nullptr;                // [P][2][kMaxValid] leading points from the cube's last DS
  int* vseg_skip = nullptr;                // [P][2][kMaxValid] 1: k_vg_merge wrote the segment
  VgSplit vgs;                             // the stack job's big-segment split (2P parents)
  float4* reg = nullptr;      // [P][capS] registered full cloud
  double* part = nullptr;     // [P][kMpSmallGrid][28] k_mp_lm_small's per-workgroup JᵀJ | Jᵀb | rows
  int* done = nullptr;        // [P] its workgroups finished (the last one runs the step)
  // the persistent one-instance L-M (k_mp_lm_stream): per workgroup and iteration parity its partial
  // sums, per workgroup its publication word (epoch << 16 | iteration + 1), the launch epoch
  // (advanced by k_mp_lm_begin)
  double* ls_part = nullptr;              // [2][kMpSmallGrid][28]
  unsigned long long* ls_flag = nullptr;  // [kMpSmallGrid]
  unsigned long long* ls_epoch = nullptr; // [1]
  double* rot = nullptr;      // [P][6] cos / sin of the TobeMapped rotation (rot_store in mp.hip)
  int* nreg = nullptr;
  // the streaming frame's map update (insertion, per-cube VoxelGrid, compaction) deferred to a side
  // stream (mp_frame's `defer`): upd_done is recorded there; the next frame, the surround cloud
  // and a reset wait for it first (upd_pending)
  hipEvent_t upd_fork = nullptr, upd_done = nullptr;
  bool upd_pending = false;
  Tuning tune;                // host-side launch choices (mp_frame)
  hipError_t sticky = hipSuccess;  // first failed HIP call of the launch sequences
  void note(hipError_t e) {
    if (sticky == hipSuccess) sticky = e;
  }
  // returns the sticky error and clears it
  hipError_t take_error() {
    const hipError_t e = sticky;
    sticky = hipSuccess;
    return e;
  }
};

inline int mp_batch_map_capacity(int cap) { return 2 * cap; }
hipError_t mp_alloc(MpBuffers& b, int P, int R, int cap_pts, int map_cap, int max_iter);  // on failure: freed, b empty
void mp_free(MpBuffers& b);
hipError_t mp_reset(MpBuffers& b, hipStream_t st);
// map_empty: the store was just reset (no L-M can run: its launches are skipped)
// before_register: called once every kernel before k_mp_register is enqueued (the streaming path
// stages the full cloud there); stack_max: the largest stack segment (corner or surf input count)
// when the host knows it, else -1
// side: an idle second stream (and two fork / join event pairs) for the frame's independent
// branches: the stack VoxelGrid beside the FromMap gather + hash builds, and the registration of the
// full cloud beside the map insertion / per-cube VoxelGrid
struct SideStream {
  hipStream_t st = nullptr;
  hipEvent_t fork[2] = {nullptr, nullptr}, join[2] = {nullptr, nullptr};
  hipEvent_t inputs_read = nullptr;  // optional: recorded once the frame has read its input clouds
};
// defer: a second stream for the map update (streaming frames): the update runs there after the
// L-M, beside the registration and the caller's downloads; the frame's pose and registered cloud do
// not wait for it (b.upd_pending until the next frame's first kernel has waited for it)
void mp_frame(MpBuffers& b, const MpInput& in, hipStream_t st, Prof* prof = nullptr, bool map_empty = false,
              const std::function<void()>& before_register = nullptr, int stack_max = -1,
              const SideStream* side = nullptr, hipStream_t defer = nullptr);
// the pending deferred map update (if any) before later work on st
void mp_wait_update(MpBuffers& b, hipStream_t st);
// imu_rp: the IMU (roll, pitch) transformUpdate blends in (nullptr = no IMU); *updated = whether
// transformUpdate ran (the caller then commits its IMU queue pointer)
int mp_stream_frame(MpBuffers& b, hipStream_t st, const loam_pose6& odom_sum, const loam_cloud_out& corner,
                    const loam_cloud_out& surf, const loam_cloud_out& full, loam_pose6* aft, loam_pose6* bef,
                    loam_cloud_out* registered, loam_stats* stats, std::string& err, Staging& pin, const StreamIo& io,
                    const float* imu_rp = nullptr, bool* updated = nullptr, hipStream_t st2 = nullptr,
                    hipEvent_t ev2 = nullptr, hipStream_t defer = nullptr);
// the same frame on clouds already on the device (src: pointers + device counts, n3: host counts)
int mp_stream_frame_dev(MpBuffers& b, hipStream_t st, const loam_pose6& odom_sum, const MpInput& src, const int* n3,
                        loam_pose6* aft, loam_pose6* bef, loam_cloud_out* registered, loam_stats* stats,
                        std::string& err, Staging& pin, const StreamIo& io, const float* imu_rp = nullptr,
                        bool* updated = nullptr, hipStream_t defer = nullptr);
// /laser_cloud_surround of the last streaming frame (instance 0): its 5x5x5 cube neighbourhood
// concatenated and VoxelGrid 0.2 (src/laserMapping.cpp:1038-1058)
int mp_stream_surround(MpBuffers& b, hipStream_t st, loam_cloud_out* out, std::string& err);
// buf: the odometry's Last buffer the frame reads (frame 1: the seed's, frame 2: TransformToEnd's)
// fprev / fcur: the scan registration outputs whose full clouds the frames register
// side: only its inputs_read event is used (the frame runs on st alone)
void mp_batch_frame1(MpBuffers& b, const OdBuffers& od, int buf, const FeatView& fprev, hipStream_t st,
                     Prof* prof = nullptr, const SideStream* side = nullptr);
void mp_batch_frame2(MpBuffers& b, const OdBuffers& od, int buf, const FeatView& fcur, hipStream_t st,
                     Prof* prof = nullptr, const SideStream* side = nullptr);
int mp_batch_download(MpBuffers& b, hipStream_t st, loam_pose6* aft, loam_stats* stats, std::string& err);
hipError_t mp_batch_iters(MpBuffers& b, hipStream_t st, int32_t* iters);

}  // namespace loam
#endif
