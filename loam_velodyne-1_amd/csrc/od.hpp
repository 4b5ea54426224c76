// Odometry / hash device buffers and kernel declarations (engine-internal).
#ifndef LOAM_OD_HPP
#define LOAM_OD_HPP

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine.hpp"

namespace loam {

// k_od_lm_stream: workgroups at most (each serves 8 association waves / their queries' rows)
constexpr int kOdLsMaxG = 128;
// per-problem float state: transform[6] | transformSum[6] | matP[36] | imu_trans[12]
#ifndef LOAM_OD_CHUNK
#define LOAM_OD_CHUNK 64
#endif
// k_od_end workgroups per problem in batches (TransformToEnd of the Last clouds)
#ifndef LOAM_OD_END_WG
#define LOAM_OD_END_WG 16  // (1024 problems: 16 / 8 / 4 measured equal once end_rot_wave took the setup)
#endif
constexpr int kOdEndWg = LOAM_OD_END_WG;
constexpr int kChunk = LOAM_OD_CHUNK;  // points per chunk box (<= 64)
__host__ __device__ inline int chunks_of(int cap) { return (cap + kChunk - 1) / kChunk; }
// the association's best-first ring windows (ring-monotone clouds) visit kSub-point sub-chunks
#ifndef LOAM_WIN_SUB
#define LOAM_WIN_SUB 32
#endif
constexpr int kSub = LOAM_WIN_SUB;
static_assert(kSub == 16 || kSub == 32 || kSub == 64, "sub-chunks of 16, 32 or 64 points");
__host__ __device__ inline int subs_of(int cap) { return (cap + kSub - 1) / kSub; }
constexpr int kOdSum = 6, kOdMatP = 12, kOdImu = 48, kOdStateFloats = 64;
// per-problem int state
enum { kIsDegenerate = 0, kIsCornerLastNum, kIsSurfLastNum, kIsIters, kIsAssoc, kIsRows, kIsQueries,
       kIsErr, kIsActive, kIsStop,
       kIsDegSteps,  // L-M updates of this frame projected by the iteration-0 degeneracy analysis (Q15)
       kIsNanSkips,  // L-M updates of this frame skipped by the NaN guard (Q16)
       kIsGathered,  // Last-cloud points the association loaded this frame (work counter)
       kIsBoxes,     // chunk boxes the association loaded this frame (work counter)
       kOdStateInts = 16 };

// read-only view of one feature set per problem (stride = elements between problems)
struct FeatView {
  const float4 *sharp, *lsharp, *flat, *lflat, *full;
  size_t sharp_stride, lsharp_stride, flat_stride, lflat_stride, full_stride;
  const int* cnt;       // 4 counts per problem at cnt[p * cnt_stride]
  int cnt_stride;
  const int* nfull_p;   // full-cloud count at nfull_p[p * nfull_stride]
  int nfull_stride;
  __device__ __forceinline__ int count(int p, int k) const { return cnt[p * cnt_stride + k]; }
  __device__ __forceinline__ int nfull(int p) const { return nfull_p[p * nfull_stride]; }
};

struct HashJob {
  const float4* pts;    // cloud of problem p at pts + p * pts_stride (+ pts_off[p * pts_off_stride])
  size_t pts_stride;
  const int* pts_off;   // optional per-problem element offset (nullptr = 0)
  int pts_off_stride;
  const int* count;     // count of problem p at (char*)count + p * count_stride_bytes
  size_t count_stride_bytes;
  int* start;           // [P][tmax + 1]
  int* fill;            // [P][tmax]
  float4* out;          // [P][pts_stride]
  int* tsize;           // [P] table size used
  int tmax;
  float inv_h;
  int shift;            // T = pow2 >= count >> shift
  float4* chunks;       // optional [P][2 * chunks_of(pts_stride)]: per 64-point chunk of the source
                        // order, (min x, y, z, min ring) and (max x, y, z, max ring)
  float4* fine = nullptr;   // optional [P][2 * subs_of(pts_stride)]: the same boxes per kSub-point sub-chunk
  uint32_t* rec = nullptr;  // optional [P][tmax]: bucket b's range packed as start | count << 19
                            // (hash_rec), kRecNone when it does not fit
  int* mono = nullptr;      // optional: mono[p * mono_stride] = 1 when the cloud's rings int(w) never
  int mono_stride = 1;      // decrease in index order (the association's window bounds rely on it)
  int* rstart = nullptr;    // optional [P][rstart_stride]: rstart[r] = first index whose ring int(w) >= r
  int rstart_stride = 0;    // (r in [0, kRingTab), n when none; meaningful for a ring-monotone cloud only)
};
constexpr int kRingTab = 66;  // rings 0..63 (n_rings <= 64) and two past the last
constexpr uint32_t kRecNone = 0xffffffffu;
LOAM_HD uint32_t hash_rec(int start, int count) {
  return start < (1 << 19) && count < (1 << 13) ? (uint32_t)start | ((uint32_t)count << 19) : kRecNone;
}

// Last-cloud buffers (Last corner / surf, fullEnd, their counts, hashes, boxes, flags): the streaming
// path alternates two, the batch step pipeline rotates three (the seed's, TransformToEnd's, a free one)
constexpr int kOdBufs = 3;

struct OdBuffers {
  int P = 0, capC = 0, capS = 0, cap_q = 0, gq = 0, tC = 0, tS = 0, max_iter = 25;
  float* state = nullptr;   // [P][kOdStateFloats] (one of state_set: batches alternate per step)
  float* state_set[3] = {nullptr, nullptr, nullptr};  // (the step pipeline's buffer slots)
  int* istate = nullptr;    // [P][kOdStateInts] (one of istate_set: batches alternate per step)
  int* istate_set[3] = {nullptr, nullptr, nullptr};
  // the streaming frame's hash build of the new Last clouds deferred to a side stream (engine
  // od_frame, tuning stream_defer): recorded there, waited for by the next frame (hash_pending)
  hipEvent_t hash_fork = nullptr, hash_done = nullptr;
  bool hash_pending = false;
  // (one problem, optional) k_od_begin first copies the state / istate here: the chain's odometry
  // may run before its scan registration's result is known, and is undone from the copy when that
  // reports an error (engine od_frame)
  float* bk_state = nullptr;
  int* bk_istate = nullptr;
  float4* lastC = nullptr;  // [kOdBufs][P][capC]
  float4* lastS = nullptr;  // [kOdBufs][P][capS]
  float4* fullEnd = nullptr;  // [kOdBufs][P][capS]
  int* nlast = nullptr;     // [P][kOdBufs][2]
  int* nfullEnd = nullptr;  // [P][kOdBufs]
  int* hC_start = nullptr;  // [kOdBufs][P][tC+1]
  int* hS_start = nullptr;  // [kOdBufs][P][tS+1]
  int* hC_fill = nullptr;   // [P][tC]
  int* hS_fill = nullptr;   // [P][tS]
  float4* hC_pts = nullptr; // [kOdBufs][P][capC]
  float4* hS_pts = nullptr; // [kOdBufs][P][capS]
  int* hC_T = nullptr;      // [kOdBufs][P]
  int* hS_T = nullptr;      // [kOdBufs][P]
  float4* cC = nullptr;     // [kOdBufs][P][2 * chunks_of(capC)] chunk boxes of Last corner
  float4* cS = nullptr;     // [kOdBufs][P][2 * chunks_of(capS)] chunk boxes of Last surf
  float4* fC = nullptr;     // [kOdBufs][P][2 * subs_of(capC)] sub-chunk boxes of Last corner (HashJob::fine)
  float4* fS = nullptr;     // [kOdBufs][P][2 * subs_of(capS)] sub-chunk boxes of Last surf
  float4* sel = nullptr;      // [P][cap_q] queries at the current transform (association rounds)
  int* ind = nullptr;         // [P][3][cap_q] association of every query (refreshed every 5th iteration)
  float4* q_cf = nullptr;     // [P][max_iter][cap_q] coefficients (zero when rejected)
  int8_t* q_ok = nullptr;     // [P][max_iter][cap_q] accepted flags
  float4* qa = nullptr;       // [P][cap_q][3] a query's associated Last points for its round (k_od_rows_mom)
  double* mom = nullptr;      // [P][10][cap_q] per-query fp64 moments of the stored rows (tuning od_moments)
  double* part = nullptr;     // [P][gq][28] per-workgroup JᵀJ | Jᵀb | rows
  int* done = nullptr;        // [P] workgroups of k_od_rows finished (the last one runs the step)
  // the persistent one-problem L-M (k_od_lm_stream): per workgroup and iteration parity its partial
  // sums, per workgroup its publication word (epoch << 16 | iteration + 1), and the launch epoch
  // (advanced by k_od_begin, so a replayed graph gets a fresh one)
  double* ls_part = nullptr;              // [2][kOdLsMaxG][28]
  unsigned long long* ls_flag = nullptr;  // [kOdLsMaxG]
  unsigned long long* ls_epoch = nullptr; // [1]
  int* mono = nullptr;        // [kOdBufs][P][2] Last corner / surf of each buffer ring-monotone (HashJob::mono)
  int* rstart = nullptr;      // [kOdBufs][P][2][kRingTab] their ring start tables (HashJob::rstart)
  Tuning tune;                // host-side launch choices (od_solve)
};

// both clouds' indexes: a workgroup per cloud for batches, a grid per cloud for P <= 4
// wide: 1024-thread workgroups (the odometry Last clouds: 0.28 -> 0.19 ms/step at batch 1024), else
// 512 (the map clouds: 0.27 -> 0.26; 1024 measured 0.31)
void hash_build_pair(const HashJob& a, const HashJob& b, int P, hipStream_t st, bool wide);

__global__ void k_od_end(OdBuffers b, FeatView f, int dst, int mode, int do_full);

hipError_t od_alloc(OdBuffers& b, int P, int R, int cap_pts, int max_iter);  // on failure: freed, b empty
void od_free(OdBuffers& b);
void od_build_hashes(const OdBuffers& b, int buf, hipStream_t st);
// od_build_hashes on `side` after the work enqueued on st so far (b.hash_pending until od_wait_hashes)
hipError_t od_build_hashes_deferred(OdBuffers& b, int buf, hipStream_t st, hipStream_t side);
hipError_t od_wait_hashes(OdBuffers& b, hipStream_t st);
// the laserOdometry L-M loop + pose accumulation for every problem against Last[last_buf]
// device_fini: the pose accumulation (k_od_fini) on the device; the streaming path does it on the host
void od_solve(const OdBuffers& b, const FeatView& f, int last_buf, hipStream_t st, Prof* prof = nullptr,
              bool device_fini = true);
// the pose accumulation alone (k_od_fini), for a caller that runs it beside TransformToEnd
void od_fini(const OdBuffers& b, const FeatView& f, hipStream_t st);

}  // namespace loam

#endif
