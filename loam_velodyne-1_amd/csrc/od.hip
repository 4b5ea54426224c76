// Laser odometry on gfx950: the laserOdometry loop body (/root/reference/src/laserOdometry.cpp:413-931)
// for a batch of independent problems.
//
//  k_hash_build   voxel-hashed CSR index of a cloud (spatial hash of 1 m cells -> buckets, counting
//                 sort).  Replaces kdtreeCornerLast / kdtreeSurfLast (:78-79, :436-437, :905-906).
//  the L-M loop (:465-828) as one launch sequence per iteration over every problem at once:
//  k_od_begin     IMU prior, whether L-M runs (:461-465)
//  k_od_assoc     every 5th iteration, one wave per query: TransformToStart, exact NN through the
//                 hash (27 cells; exhaustive fallback when the best match is farther than one cell),
//                 then the ring-window scans of :486-523 / :598-645 as 64-wide chunks with a
//                 ballot for the break and a (distance, scan order) min-reduction = the
//                 reference's sequential first-minimum
//  k_od_rows      lane per query: residual + weight of this iteration stored per (iteration, query)
//                 (the row order of the reference's append, Q12), J of every row accumulated so far
//                 at the current transform, JᵀJ / Jᵀb partial sums in fp64
//                 the last workgroup of a problem to finish then sums the partials in a fixed
//                 order and runs the 6x6 QR solve / iteration-0 degeneracy analysis on one lane,
//                 NaN guard, convergence test (od_step)
//  k_od_fini      pose accumulation (:830-856)
//  k_od_end       TransformToEnd of lessSharp / lessFlat / full (:875-891) into the next Last clouds.
#include "dev_common.hpp"
#include "od.hpp"
#include "pose_math.hpp"

using namespace loamdev;

// batch-size launch choices (k_od_rows_small / k_od_rows<true> / k_od_assoc grid): the
// context's Tuning (engine.hpp), OdBuffers::tune
// (measured at batch 128: k_od_rows<true> rows + step 0.67 -> 0.62 ms/step, whole step unchanged;
// 1024 slower)

// diagnostic builds: count only one phase's gathered points in od_assoc_gathered (1: the 27 cells,
// 2: the chunk fallback beyond one cell, 3: the ring windows); 0 (product): all
// LOAM_ASSOC_SKIP (timing attribution builds only, results wrong): 1 no ring windows, 2 no chunk
// fallback of the nearest-neighbour search, 3 neither
#ifndef LOAM_ASSOC_SKIP
#define LOAM_ASSOC_SKIP 0
#endif
#ifndef LOAM_ASSOC_PHASE
#define LOAM_ASSOC_PHASE 0
#endif
#if (LOAM_ASSOC_SKIP != 0 || LOAM_ASSOC_PHASE != 0) && !defined(LOAM_EXPERIMENT_BUILD)
#error "LOAM_ASSOC_SKIP / LOAM_ASSOC_PHASE are diagnostic (wrong results / partial counters): tools/build_variant.sh only"
#endif

namespace loam {
#ifdef LOAM_PHASES
__device__ PhaseAcc g_ph_od = {~0ull, 0ull, 0ull, {{0}}};
#endif


namespace {

constexpr int kOdThreads = 256;
constexpr int kOdWaves = kOdThreads / 64;
// k_od_assoc: one wave (query) per workgroup, so a finished wave's slot is not held for its
// workgroup's slowest query (ms/step at batch 1024: 256 threads -> 2.91, 128 -> 2.88, 64 -> 2.82-2.85)
constexpr int kAsThreads = 64, kAsWaves = kAsThreads / 64;

LOAM_D loampose::Imu load_imu(const float* st) {
  loampose::Imu m;
  const float* q = st + kOdImu;
  m.pitchStart = q[0]; m.yawStart = q[1]; m.rollStart = q[2];
  m.pitchLast = q[3]; m.yawLast = q[4]; m.rollLast = q[5];
  m.shiftX = q[6]; m.shiftY = q[7]; m.shiftZ = q[8];
  m.veloX = q[9]; m.veloY = q[10]; m.veloZ = q[11];
  return m;
}

}  // namespace

// ---------------------------------------------------------------- voxel hash build
// One workgroup per cloud: T = pow2 >= count >> shift (clamped to [64, tmax]) buckets — a 1 m
// cell holds several points, so even two points per bucket (shift 1) leaves distinct neighbouring
// cells rarely sharing a bucket — CSR start[T+1], points re-ordered by bucket with their source index in .w
// (bit pattern; for the odometry clouds index | ring << 24).  Bucket counters live in LDS up to
// kHashLds buckets, in global memory beyond.
constexpr int kHashLds = 8192;


// counting sort of the cloud's points by bucket; fill = LDS (LDS true) or this cloud's global
// counters (read back with atomic loads: the counts were made by L2 atomics)
template <int NT, bool LDS>
LOAM_D void hash_sort(const HashJob& j, const float4* pts, int n, int T, int* start, float4* out, int* fill,
                      int* scratch, uint32_t* rec) {
  const int tid = threadIdx.x;
  auto ld = [&](int b) {
    if constexpr (LDS) return fill[b];
    else return __hip_atomic_load(&fill[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  for (int b = tid; b < T; b += NT) fill[b] = 0;
  if (!LDS) __threadfence();
  __syncthreads();
  for (int i = tid; i < n; i += NT) {
    const float4 a = pts[i];
    uint32_t h = cell_hash(cell_of(a.x, j.inv_h), cell_of(a.y, j.inv_h), cell_of(a.z, j.inv_h)) & (T - 1);
    atomicAdd(&fill[h], 1);
  }
  if (!LDS) __threadfence();
  __syncthreads();
  // exclusive scan of fill[0..T) into start: contiguous chunk per thread
  const int per = (T + NT - 1) / NT;
  const int b0 = tid * per, b1 = min(T, b0 + per);
  int local = 0;
  for (int b = b0; b < b1; ++b) local += ld(b);
  int tot;
  int run = block_excl_scan<NT>(local, scratch, tot);
  if constexpr (LDS) {
    // the bucket starts into LDS, then start / rec written bucket-consecutive across the lanes
    // (a thread's own run of buckets would make every store a 64-line scatter)
    for (int b = b0; b < b1; ++b) {
      const int c = fill[b];
      fill[b] = run;
      run += c;
    }
    __syncthreads();
    for (int b = tid; b < T; b += NT) {
      const int s0 = fill[b], s1 = b + 1 < T ? fill[b + 1] : tot;
      start[b] = s0;
      if (rec) rec[b] = hash_rec(s0, s1 - s0);
    }
  } else {
    for (int b = b0; b < b1; ++b) {
      const int c = ld(b);
      start[b] = run;
      if (rec) rec[b] = hash_rec(run, c);
      __hip_atomic_store(&fill[b], run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      run += c;
    }
  }
  if (tid == 0) start[T] = tot;
  if (!LDS) __threadfence();
  __syncthreads();
  for (int i = tid; i < n; i += NT) {
    const float4 a = pts[i];
    uint32_t h = cell_hash(cell_of(a.x, j.inv_h), cell_of(a.y, j.inv_h), cell_of(a.z, j.inv_h)) & (T - 1);
    int pos = atomicAdd(&fill[h], 1);
    // odometry clouds (chunk boxes built): the ring rides in the top byte, so the nearest
    // neighbour's ring needs no extra load (wave_hash_nn)
    const int tag = j.chunks ? (i | ((int)a.w << 24)) : i;
    out[pos] = make_float4(a.x, a.y, a.z, __int_as_float(tag));
  }
}

// the chunk boxes (min / max of x, y, z and of the ring int(intensity)) of points [0, n) in
// CHK-point chunks, 64 / CHK chunks per wave step; wave w0 of nw waves
template <int CHK = kChunk>
LOAM_D void chunk_boxes(const float4* pts, int n, float4* ch, int w0, int nw) {
  const int lane = lane_id();
  constexpr int PER = 64 / CHK;
  const int nch = (n + CHK - 1) / CHK;
  for (int c0 = w0 * PER; c0 < nch; c0 += nw * PER) {
    const int c = c0 + lane / CHK;
    const float4 a = pts[min(c * CHK + lane % CHK, n - 1)];
    const float r = (float)(int)a.w;
    float4 lo = make_float4(a.x, a.y, a.z, r), hi = lo;
#pragma unroll
    for (int o = CHK / 2; o > 0; o >>= 1) {
      lo.x = fminf(lo.x, __shfl_xor(lo.x, o, 64)); lo.y = fminf(lo.y, __shfl_xor(lo.y, o, 64));
      lo.z = fminf(lo.z, __shfl_xor(lo.z, o, 64)); lo.w = fminf(lo.w, __shfl_xor(lo.w, o, 64));
      hi.x = fmaxf(hi.x, __shfl_xor(hi.x, o, 64)); hi.y = fmaxf(hi.y, __shfl_xor(hi.y, o, 64));
      hi.z = fmaxf(hi.z, __shfl_xor(hi.z, o, 64)); hi.w = fmaxf(hi.w, __shfl_xor(hi.w, o, 64));
    }
    if (lane % CHK == 0 && c < nch) {
      ch[2 * c] = lo;
      ch[2 * c + 1] = hi;
    }
  }
}

// the ring start table of a ring-monotone cloud (HashJob::rstart): point i (of threads t0, t0 + nt,
// ...) opens the rings above its predecessor's up to its own; the last point closes the rest
LOAM_D void ring_starts(const HashJob& j, const float4* pts, int n, int p, int t0, int nt) {
  int* rs = j.rstart + (size_t)p * j.rstart_stride;
  auto ring = [&](int i) { return min(max((int)pts[i].w, 0), kRingTab - 1); };
  if (n == 0 && t0 < kRingTab)
    for (int r = t0; r < kRingTab; r += nt) rs[r] = 0;
  for (int i = t0; i < n; i += nt) {
    const int r = ring(i), rp = i > 0 ? ring(i - 1) : -1;
    for (int rr = rp + 1; rr <= r; ++rr) rs[rr] = i;
    if (i == n - 1)
      for (int rr = r + 1; rr < kRingTab; ++rr) rs[rr] = n;
  }
}

struct HashPair {
  HashJob j[2];
};

// both clouds' indexes in one launch: blockIdx.y selects the job (the two are independent)
template <int NT>
__global__ __launch_bounds__(NT) void k_hash_build(HashPair hp) {
  const HashJob& j = hp.j[blockIdx.y];
  const int p = blockIdx.x, tid = threadIdx.x;
  const int n = *(const int*)((const char*)j.count + (size_t)p * j.count_stride_bytes);
  const float4* pts = j.pts + (size_t)p * j.pts_stride + (j.pts_off ? j.pts_off[p * j.pts_off_stride] : 0);
  int* start = j.start + (size_t)p * (j.tmax + 1);
  float4* out = j.out + (size_t)p * j.pts_stride;
  __shared__ int scratch[NT / 64 + 1];
  __shared__ int lfill[kHashLds];
  const int m = n >> j.shift;
  int T = next_pow2(m > 64 ? m : 64);
  if (T > j.tmax) T = j.tmax;
  if (tid == 0) j.tsize[p] = T;
  uint32_t* rec = j.rec ? j.rec + (size_t)p * j.tmax : nullptr;
  if (T <= kHashLds) hash_sort<NT, true>(j, pts, n, T, start, out, lfill, scratch, rec);
  else hash_sort<NT, false>(j, pts, n, T, start, out, j.fill + (size_t)p * j.tmax, scratch, rec);
  if (j.chunks)  // chunk boxes of the source order
    chunk_boxes(pts, n, j.chunks + (size_t)p * 2 * chunks_of((int)j.pts_stride), tid >> 6, NT / 64);
  if (j.fine) chunk_boxes<kSub>(pts, n, j.fine + (size_t)p * 2 * subs_of((int)j.pts_stride), tid >> 6, NT / 64);
  if (j.mono) {  // rings non-decreasing in index order (one flag per cloud: no atomics)
    bool bad = false;
    for (int i = tid + 1; i < n; i += NT) bad |= (int)pts[i].w < (int)pts[i - 1].w;
    bad = __syncthreads_or(bad);
    if (tid == 0) j.mono[(size_t)p * j.mono_stride] = bad ? 0 : 1;
  }
  if (j.rstart) ring_starts(j, pts, n, p, tid, NT);
}

// ---- the same index built by many workgroups per cloud (small batches: streaming, config 2).  One
// workgroup per cloud left a few CUs busy for 40-60 us per map; here a grid per cloud zeroes the
// bucket counters, counts with global atomics, one workgroup scans, and the grid scatters.  The
// order of points inside a bucket differs from the single-workgroup build (both are atomic
// orders); no consumer depends on it (every search breaks ties on the source index).
constexpr int kHashGrid = 32;  // workgroups per cloud

LOAM_D int hash_table_size(const HashJob& j, int n) {
  const int m = n >> j.shift;
  const int T = next_pow2(m > 64 ? m : 64);
  return T > j.tmax ? j.tmax : T;
}
LOAM_D int hash_count_of(const HashJob& j, int p) {
  return *(const int*)((const char*)j.count + (size_t)p * j.count_stride_bytes);
}

__global__ __launch_bounds__(256) void k_hash_zero(HashPair hp) {
  const HashJob& j = hp.j[blockIdx.z];
  const int p = blockIdx.y;
  const int T = hash_table_size(j, hash_count_of(j, p));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    j.tsize[p] = T;
    if (j.mono) j.mono[(size_t)p * j.mono_stride] = 1;  // (k_hash_count clears it on a ring drop)
  }
  int* fill = j.fill + (size_t)p * j.tmax;
  for (int b = blockIdx.x * 256 + threadIdx.x; b < T; b += gridDim.x * 256) fill[b] = 0;
}

__global__ __launch_bounds__(256) void k_hash_count(HashPair hp) {
  const HashJob& j = hp.j[blockIdx.z];
  const int p = blockIdx.y, tid = threadIdx.x;
  const int n = hash_count_of(j, p);
  const int T = hash_table_size(j, n);
  const float4* pts = j.pts + (size_t)p * j.pts_stride + (j.pts_off ? j.pts_off[p * j.pts_off_stride] : 0);
  int* fill = j.fill + (size_t)p * j.tmax;
  for (int i = blockIdx.x * 256 + tid; i < n; i += gridDim.x * 256) {
    const float4 a = pts[i];
    const uint32_t h = cell_hash(cell_of(a.x, j.inv_h), cell_of(a.y, j.inv_h), cell_of(a.z, j.inv_h)) & (T - 1);
    atomicAdd(&fill[h], 1);
  }
  if (j.chunks)  // chunk boxes of the source order (as k_hash_build)
    chunk_boxes(pts, n, j.chunks + (size_t)p * 2 * chunks_of((int)j.pts_stride), blockIdx.x * 4 + (tid >> 6),
                gridDim.x * 4);
  if (j.fine)
    chunk_boxes<kSub>(pts, n, j.fine + (size_t)p * 2 * subs_of((int)j.pts_stride), blockIdx.x * 4 + (tid >> 6),
                      gridDim.x * 4);
  if (j.mono) {
    bool bad = false;
    for (int i = blockIdx.x * 256 + tid + 1; i < n; i += gridDim.x * 256) bad |= (int)pts[i].w < (int)pts[i - 1].w;
    if (bad) j.mono[(size_t)p * j.mono_stride] = 0;
  }
  if (j.rstart) ring_starts(j, pts, n, p, blockIdx.x * 256 + tid, gridDim.x * 256);
}

// exclusive scan of the counters into start (and back into fill as the scatter's cursors)
__global__ __launch_bounds__(1024) void k_hash_scan(HashPair hp) {
  const HashJob& j = hp.j[blockIdx.z];
  const int p = blockIdx.y, tid = threadIdx.x;
  const int n = hash_count_of(j, p);
  const int T = hash_table_size(j, n);
  int* fill = j.fill + (size_t)p * j.tmax;
  int* start = j.start + (size_t)p * (j.tmax + 1);
  uint32_t* rec = j.rec ? j.rec + (size_t)p * j.tmax : nullptr;
  __shared__ int scratch[32];
  const int per = (T + 1023) / 1024;
  const int b0 = tid * per, b1 = min(T, b0 + per);
  if (per % 4 == 0 && per <= 64 && T % 1024 == 0) {  // uniform: every run is full
    // the thread's run as up to sixteen 16-B loads, all in flight (T is a power of two: per divides it)
    constexpr int kV = 16;
    int4 v[kV];
    const int4* f4 = (const int4*)(fill + b0);
    const int nv = per / 4;
#pragma unroll
    for (int k = 0; k < kV; ++k)
      if (k < nv) v[k] = f4[k];
    int local = 0;
#pragma unroll
    for (int k = 0; k < kV; ++k)
      if (k < nv) local += v[k].x + v[k].y + v[k].z + v[k].w;
    int tot;
    int run = block_excl_scan<1024>(local, scratch, tot);
    int4* o4 = (int4*)(fill + b0);
#pragma unroll
    for (int k = 0; k < kV; ++k)
      if (k < nv) {
        int4 r;
        r.x = run; run += v[k].x;
        r.y = run; run += v[k].y;
        r.z = run; run += v[k].z;
        r.w = run; run += v[k].w;
        o4[k] = r;
        start[b0 + 4 * k] = r.x;
        start[b0 + 4 * k + 1] = r.y;
        start[b0 + 4 * k + 2] = r.z;
        start[b0 + 4 * k + 3] = r.w;
        if (rec)
          *(uint4*)(rec + b0 + 4 * k) = make_uint4(hash_rec(r.x, v[k].x), hash_rec(r.y, v[k].y),
                                                   hash_rec(r.z, v[k].z), hash_rec(r.w, v[k].w));
      }
    if (tid == 0) start[T] = tot;
    return;
  }
  int local = 0;
  for (int b = b0; b < b1; ++b) local += fill[b];
  int tot;
  int run = block_excl_scan<1024>(local, scratch, tot);
  for (int b = b0; b < b1; ++b) {
    const int c = fill[b];
    start[b] = run;
    if (rec) rec[b] = hash_rec(run, c);
    fill[b] = run;
    run += c;
  }
  if (tid == 0) start[T] = tot;
}

__global__ __launch_bounds__(256) void k_hash_scatter(HashPair hp) {
  const HashJob& j = hp.j[blockIdx.z];
  const int p = blockIdx.y;
  const int n = hash_count_of(j, p);
  const int T = hash_table_size(j, n);
  const float4* pts = j.pts + (size_t)p * j.pts_stride + (j.pts_off ? j.pts_off[p * j.pts_off_stride] : 0);
  int* fill = j.fill + (size_t)p * j.tmax;
  float4* out = j.out + (size_t)p * j.pts_stride;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const float4 a = pts[i];
    const uint32_t h = cell_hash(cell_of(a.x, j.inv_h), cell_of(a.y, j.inv_h), cell_of(a.z, j.inv_h)) & (T - 1);
    const int pos = atomicAdd(&fill[h], 1);
    const int tag = j.chunks ? (i | ((int)a.w << 24)) : i;
    out[pos] = make_float4(a.x, a.y, a.z, __int_as_float(tag));
  }
}

void hash_build_pair(const HashJob& a, const HashJob& b, int P, hipStream_t st, bool wide) {
  if (P > 4) {  // batches: a workgroup per cloud fills the chip
    HashPair hp;
    hp.j[0] = a;
    hp.j[1] = b;
    if (wide) hipLaunchKernelGGL(k_hash_build<1024>, dim3(P, 2), dim3(1024), 0, st, hp);
    else hipLaunchKernelGGL(k_hash_build<512>, dim3(P, 2), dim3(512), 0, st, hp);
    return;
  }
  HashPair hp;
  hp.j[0] = a;
  hp.j[1] = b;
  hipLaunchKernelGGL(k_hash_zero, dim3(kHashGrid, P, 2), dim3(256), 0, st, hp);
  hipLaunchKernelGGL(k_hash_count, dim3(kHashGrid, P, 2), dim3(256), 0, st, hp);
  hipLaunchKernelGGL(k_hash_scan, dim3(1, P, 2), dim3(1024), 0, st, hp);
  hipLaunchKernelGGL(k_hash_scatter, dim3(kHashGrid, P, 2), dim3(256), 0, st, hp);
}

namespace {


// lower bound of the float squared distance from s to any point of the box [lo, hi] (monotone
// rounding of the same expression as sqdist)
LOAM_D float box_d2(const float4& lo, const float4& hi, const float4& s) {
  const float gx = fmaxf(fmaxf(lo.x - s.x, s.x - hi.x), 0.0f);
  const float gy = fmaxf(fmaxf(lo.y - s.y, s.y - hi.y), 0.0f);
  const float gz = fmaxf(fmaxf(lo.z - s.z, s.z - hi.z), 0.0f);
  return sqdist(gx, gy, gz, 0.0f, 0.0f, 0.0f);
}

// j (ring r) belongs to the window set of a query whose nearest point is c (ring scan): the points
// the forward walk c+1 .. fwd_end-1 and the backward walk c-1 .. 0 visit before their stops, of the
// wanted category (corner: the other rings; surf: same = the same / lower ring forward and the same /
// higher ring backward, else the other rings).  Exact for a ring-monotone cloud (HashJob::mono),
// where every point of rings scan - 2 .. scan + 2 on the walk's side precedes the stop.
LOAM_D bool window_member(int j, int r, int c, int scan, int fwd_end, bool corner, bool same) {
  if (j > c) return j < fwd_end && r <= scan + 2 && (corner ? r > scan : (same ? r <= scan : r > scan));
  return j < c && r >= scan - 2 && (corner ? r < scan : (same ? r >= scan : r < scan));
}

// bounds of the window minima known before the walks (squared distances of members, or 25)
struct WinBound {
  float same = 25.0f, other = 25.0f;
};

// exact nearest neighbour of q among the hashed cloud (wave-cooperative), as far as it matters:
// returns the packed (float distance bits << 32 | index << 8 | ring) minimum (ties on the index,
// as before: the ring is a function of the point), or ~0 when no point lies
// closer than 5 m (the callers reject a nearest neighbour at >= 25 m², :481, :594).  First the
// 27 cells around q (cells whose box lies >= h away skipped); if the best is >= h, the chunk
// boxes of the whole cloud closer than 5 m.  `cells` = per-wave LDS scratch of 64 ints.
// bound: the squared distance of a known point of the cloud (a seed), or above 25: cells and chunks
// whose box lies beyond it cannot hold the minimum (which is <= the seed's) and are skipped
// kind 0 / 1 (corner / surf, 1 m cells only; -1: none) with mono: when the nearest point lies in the
// 27 cells, the cells' points that belong to its window sets (window_member, fwd_end) bound the
// window minima (wb): a chunk beyond such a member cannot hold the minimum.
LOAM_D uint64_t wave_hash_nn(const int* start, const float4* hp, int T, const float4* cloud, const float4* ch,
                             int n, float h, float inv_h, float4 q, float bound, int* cells, int& wpts, int& wbox,
                             int kind = -1, int fwd_end = 0, bool mono = false, WinBound* wb = nullptr) {
  const int lane = lane_id();
  const int cx = cell_of(q.x, inv_h), cy = cell_of(q.y, inv_h), cz = cell_of(q.z, inv_h);
  int bucket = -1, b0 = 0, cnt = 0;
  if (lane < 27 && T > 0) {
    const int dx = lane % 3 - 1, dy = (lane / 3) % 3 - 1, dz = lane / 9 - 1;
    const float4 lo = make_float4((float)(cx + dx) * h, (float)(cy + dy) * h, (float)(cz + dz) * h, 0.0f);
    const float4 hi = make_float4((float)(cx + dx + 1) * h, (float)(cy + dy + 1) * h, (float)(cz + dz + 1) * h, 0.0f);
    const float bd = box_d2(lo, hi, q);
    if (h != 1.0f || (bd < 1.0f && bd <= bound)) {
      bucket = (int)(cell_hash(cx + dx, cy + dy, cz + dz) & (uint32_t)(T - 1));
      const int2 rg = load_pair(start + bucket);
      b0 = rg.x;
      cnt = rg.y - b0;
      LOAM_CHECK(b0 >= 0 && cnt >= 0 && b0 + cnt <= n, b0, cnt);
    }
  }
  // (two of the 27 cells may share a bucket: its points are then offered twice, which does not
  // change a minimum)
  const int incl = wave_incl_scan_x(cnt);
  const int total = __builtin_amdgcn_readlane(incl, 63);
  if (LOAM_ASSOC_PHASE == 0 || LOAM_ASSOC_PHASE == 1) wpts += total;
  if (lane < 32) { cells[lane] = lane < 27 ? incl - cnt : 0x7fffffff; cells[32 + lane] = b0; }
  __builtin_amdgcn_wave_barrier();
  uint64_t best = ~0ull;
  auto cand = [&](int t) {
    int k = 0;  // last cell whose prefix is <= t (binary search over 32 entries)
#pragma unroll
    for (int step = 16; step > 0; step >>= 1)
      if (cells[k + step] <= t) k += step;
    LOAM_CHECK(cells[32 + k] + (t - cells[k]) < n && cells[32 + k] >= 0, cells[32 + k] + (t - cells[k]), n);
    return hp[cells[32 + k] + (t - cells[k])];
  };
  float4 a0 = make_float4(0, 0, 0, 0);  // the lane's first candidate, kept for the window bounds
  for (int t = lane; t < total; t += 64) {
    const float4 a = cand(t);
    if (t == lane) a0 = a;
    const float d = sqdist(a.x, a.y, a.z, q.x, q.y, q.z);
    const uint32_t tag = (uint32_t)__float_as_int(a.w);  // index | ring << 24
    const uint64_t key = ((uint64_t)fkey(d) << 32) | ((tag & 0xffffffu) << 8) | (tag >> 24);
    best = key < best ? key : best;
  }
  best = wave_min_u64_x(best);
  __builtin_amdgcn_wave_barrier();
  if (best != ~0ull && __uint_as_float((uint32_t)(best >> 32)) < h * h) {
    if (kind >= 0 && mono && D(__uint_as_float((uint32_t)(best >> 32))) < 25) {
      const int c = (int)((uint32_t)best >> 8), scan = (int)((uint32_t)best & 255u);
      float ms = 3.4e38f, mo = 3.4e38f;
      for (int t = lane; t < total; t += 64) {
        const float4 a = t == lane ? a0 : cand(t);
        const uint32_t tag = (uint32_t)__float_as_int(a.w);
        const int j = (int)(tag & 0xffffffu), r = (int)(tag >> 24);
        const float d = sqdist(a.x, a.y, a.z, q.x, q.y, q.z);
        if (kind == 0) {
          if (window_member(j, r, c, scan, fwd_end, true, false)) mo = fminf(mo, d);
        } else if (window_member(j, r, c, scan, fwd_end, false, true)) {
          ms = fminf(ms, d);
        } else if (window_member(j, r, c, scan, fwd_end, false, false)) {
          mo = fminf(mo, d);
        }
      }
      wb->same = fminf(wb->same, wave_min_f_x(ms));
      wb->other = fminf(wb->other, wave_min_f_x(mo));
    }
    return best;
  }
  if (LOAM_ASSOC_SKIP & 2) return best;
  // farther than one cell: the chunks of the whole cloud that may hold a point closer than 5 m
  best = ~0ull;
  const int nch = (n + kChunk - 1) / kChunk;
  for (int k0 = 0; k0 < nch; k0 += 64) {
    const int k = k0 + lane;
    float bd = 0.0f;
    if (k < nch) bd = box_d2(ch[2 * k], ch[2 * k + 1], q);
    const bool need = k < nch && bd < 25.0f && bd <= bound;
    uint64_t nb = __ballot(need);
    wbox += min(64, nch - k0);
    while (nb) {
      const int c = k0 + __ffsll((unsigned long long)nb) - 1;
      nb &= nb - 1;
      if (LOAM_ASSOC_PHASE == 0 || LOAM_ASSOC_PHASE == 2) wpts += min(kChunk, n - c * kChunk);
      const int t = c * kChunk + lane;
      if (lane < kChunk && t < n) {
        const float4 a = cloud[t];
        const float d = sqdist(a.x, a.y, a.z, q.x, q.y, q.z);
        const uint64_t key = ((uint64_t)fkey(d) << 32) | ((uint32_t)t << 8) | (uint32_t)(int)a.w;
        best = key < best ? key : best;
      }
    }
  }
  return wave_min_u64_x(best);
}

// One direction of a ring-window scan (:486-523 / :598-645) over the cloud L from c (exclusive):
// dir = +1 walks c+1 .. end-1, dir = -1 walks c-1 .. 0, stopping at the first point whose ring
// lies beyond scan +- 2.5.  `f(j, a, d)` is called by the lane holding point j (before the stop)
// with d < 25.  Whole 64-point chunks whose box is >= 5 m from sel are skipped; a chunk that may
// hold the stop is always examined.
// bs / bo: bounds of the same-ring / other-ring minima (squared distances of known members, or 25;
// bs < 0: no same-ring minimum is taken, the corner walk): a chunk is needed only when its box may
// beat the bound of a category its ring range [lo.w, hi.w] can hold
#ifndef LOAM_WIN_INFLIGHT
#define LOAM_WIN_INFLIGHT 1  // (measured k_od_assoc ms/step at batch 1024: 1 -> 2.81, 2 -> 2.80, 3 -> 3.01)
#endif
constexpr int kWinInFlight = LOAM_WIN_INFLIGHT;
template <typename F>
LOAM_D void wave_window(const float4* L, const float4* ch, int c, int end, int dir, int scan, float4 sel, float bs,
                        float bo, int& wpts, int& wbox, F f) {
  const int lane = lane_id();
  // int(intensity) > scan + 2.5 (double) <=> r > scan + 2 for integers (and < scan - 2.5 <=> < scan - 2)
  auto stop_ring = [&](int r) { return dir > 0 ? r > scan + 2 : r < scan - 2; };
  // the points [j0 .. j0 + dir * (cnt - 1)], lane k holding a = point j0 + dir * k; true when the
  // stop was met
  auto scan_pts = [&](int j0, int cnt, float4 a) {
    if (LOAM_ASSOC_PHASE == 0 || LOAM_ASSOC_PHASE == 3) wpts += cnt;
    const int j = j0 + dir * lane;
    const bool inr = lane < cnt;
    const int r = (int)a.w;
    const uint64_t mb = __ballot(inr && stop_ring(r));
    const int limit = mb ? __ffsll((unsigned long long)mb) - 1 : 64;
    if (inr && lane < limit) {
      const float d = sqdist(a.x, a.y, a.z, sel.x, sel.y, sel.z);
      if (d < 25) f(j, r, d);
    }
    return mb != 0;
  };
  // up to kWinInFlight of the window's needed chunks at once (their loads in flight together).  Only
  // the last needed chunk of a 64-box step can hold the stop (it is the first box whose ring range
  // reaches past scan +- 2), and every minimum is keyed by (distance, walk position), so taking them
  // together visits the same points and keeps the same minima as one at a time.
  auto run_set = [&](uint64_t& nb, int kbase, int ksign, int jofs) {
    bool stopped = false;
    while (nb && !stopped) {
      int j0[kWinInFlight], cn[kWinInFlight];
      float4 a[kWinInFlight];
#pragma unroll
      for (int u = 0; u < kWinInFlight; ++u) {
        cn[u] = 0;
        j0[u] = 0;
        if (nb) {
          const int kk = kbase + ksign * (__ffsll((unsigned long long)nb) - 1);
          nb &= nb - 1;
          j0[u] = kk * kChunk + jofs;
          cn[u] = dir > 0 ? min(kChunk, end - kk * kChunk) : kChunk;
        }
        const int j = j0[u] + dir * lane;
        if (lane < cn[u]) LOAM_CHECK(j >= 0 && (dir < 0 ? j < c : j < end), j, end);
        a[u] = lane < cn[u] ? L[j] : make_float4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kWinInFlight; ++u)
        if (cn[u] && !stopped) stopped = scan_pts(j0[u], cn[u], a[u]);
    }
    return stopped;
  };
  // examines points [j0 .. j0 + dir * (cnt - 1)]; true when the stop was met
  auto run = [&](int j0, int cnt) {
    const int j = j0 + dir * lane;
    const bool inr = lane < cnt;
    if (inr) LOAM_CHECK(j >= 0 && (dir < 0 ? j < c : j < end), j, end);
    return scan_pts(j0, cnt, inr ? L[j] : make_float4(0, 0, 0, 0));
  };

  if (dir > 0) {
    int j = c + 1;
    const int hend = min(end, (j + kChunk - 1) & ~(kChunk - 1));
    if (j < hend && run(j, hend - j)) return;
    j = max(j, hend);
    while (j < end) {
      const int k = (j / kChunk) + lane;
      const bool v = k * kChunk < end;
      wbox += min(64, (end - j + kChunk - 1) / kChunk);
      float4 lo = make_float4(0, 0, 0, 0), hi = lo;
      if (v) { lo = ch[2 * k]; hi = ch[2 * k + 1]; }
      const uint64_t mc = __ballot(v && stop_ring((int)hi.w));
      const int limit = mc ? __ffsll((unsigned long long)mc) - 1 : 63;
      const float bd = box_d2(lo, hi, sel);
      // forward: the same category is ring <= scan, the other ring > scan
      const bool need = bd < 25.0f && ((bd <= bs && (int)lo.w <= scan) || (bd <= bo && (int)hi.w > scan));
      uint64_t nb = __ballot(v && lane <= limit && need);
      run_set(nb, j / kChunk, +1, 0);
      if (mc) return;
      j += 64 * kChunk;
    }
  } else {
    int j = c - 1;
    if (j < 0) return;
    const int hstart = j & ~(kChunk - 1);
    if (run(j, j - hstart + 1)) return;
    int kt = hstart / kChunk - 1;  // next chunk (descending)
    while (kt >= 0) {
      const int k = kt - lane;
      const bool v = k >= 0;
      wbox += min(64, kt + 1);
      float4 lo = make_float4(0, 0, 0, 0), hi = lo;
      if (v) { lo = ch[2 * k]; hi = ch[2 * k + 1]; }
      const uint64_t mc = __ballot(v && stop_ring((int)lo.w));
      const int limit = mc ? __ffsll((unsigned long long)mc) - 1 : 63;
      const float bd = box_d2(lo, hi, sel);
      // backward: the same category is ring >= scan, the other ring < scan
      const bool need = bd < 25.0f && ((bd <= bs && (int)hi.w >= scan) || (bd <= bo && (int)lo.w < scan));
      uint64_t nb = __ballot(v && lane <= limit && need);
      run_set(nb, kt, -1, kChunk - 1);
      if (mc) return;
      kt -= 64;
    }
  }
}

// The ring windows of a ring-monotone Last cloud (HashJob::mono) as index ranges: the walks of
// :486-523 / :598-645 from the nearest point c (ring scan) visit, before their stops, exactly the points
// of [rs[scan - 2], c) backward and (c, min(fwd_end, rs[scan + 3])) forward, and a point's category is
// its ring: the same ring (surf min2: j > c ring <= scan, j < c ring >= scan) is [rs[scan], rs[scan + 1]),
// the rest are the other rings (corner, surf min3).  Each minimum is keyed by (distance, walk
// position) like the walks', so it is found by visiting the window's kSub-point sub-chunks (64 / kSub
// per wave step, in index order) while their boxes may still hold a point at or below a wanted
// category's bound — the previous round's choice when it is a member, the cells' members (wb, first
// round), then the minima so far: exact, in a few wave steps.
// fb: the cloud's kSub-point sub-chunk boxes; rs: its ring start table (LDS).  want_same: the surf min2 category is taken (corner: no).
// best2 / best3 in and out: the keys ((distance bits << 32) | walk position), ~0 for none; keys at
// or above 25 m² never count (:491, :602).
#ifndef LOAM_WIN_WB
#define LOAM_WIN_WB 0  // the first round's window bounds from the nearest neighbour's cells (wave_hash_nn):
                       // its second pass over the cells cost more than the sub-chunks it saved
                       // (k_od_assoc at 1024: 2.42 with, 2.35 without)
#endif
#ifndef LOAM_WIN_TIGHTEN
#define LOAM_WIN_TIGHTEN 0  // bounds tightened after every wave step: 0 never (the seeds' / cells' only),
#endif                      // 1 always, 2 in the first (unseeded) round

LOAM_D void wave_window_mono(const float4* L, const float4* fb, const int* rs, int c, int scan, int fwd_end,
                             float4 sel, bool want_same, const WinBound& wb, bool tighten, uint64_t& best2,
                             uint64_t& best3, int& wpts, int& wbox) {
  constexpr int PER = 64 / kSub;            // sub-chunks visited per wave step
  constexpr int BPL = kSub == 16 ? 2 : 1;   // boxes per lane per box step
  const int lane = lane_id();
  const int w0 = rs[max(scan - 2, 0)], rs0 = rs[scan], rs1 = rs[scan + 1];
  const int w1 = max(min(fwd_end, rs[min(scan + 3, kRingTab - 1)]), c + 1);
  // the lane's keys (reduced once at the end) and the categories' distance bounds (wave-uniform):
  // the seeds', the cells' (wb), 25
  uint64_t k2 = best2, k3 = best3;
  float d2 = fminf(wb.same, __uint_as_float((uint32_t)(best2 >> 32)));
  float d3 = fminf(wb.other, __uint_as_float((uint32_t)(best3 >> 32)));
  d2 = fminf(d2, 25.0f);
  d3 = fminf(d3, 25.0f);
  const int k0 = w0 / kSub, k1 = (w1 - 1) / kSub;  // sub-chunks overlapping [w0, w1)
  for (int g = k0; g <= k1; g += 64 * BPL) {
    wbox += min(64 * BPL, k1 - g + 1);
    float bd[BPL];
    bool hs[BPL], ho[BPL];
    uint64_t live[BPL];
#pragma unroll
    for (int u = 0; u < BPL; ++u) {
      const int k = g + u * 64 + lane;
      bd[u] = 3.4e38f;
      hs[u] = ho[u] = false;
      if (k <= k1) {
        bd[u] = box_d2(fb[2 * k], fb[2 * k + 1], sel);
        const int lo = max(k * kSub, w0), hi = min(k * kSub + kSub, w1);
        hs[u] = want_same && max(lo, rs0) < min(hi, rs1);
        ho[u] = lo < rs0 || hi > rs1;
      }
      live[u] = ~0ull;
    }
    while (true) {
      // the boxes that may still hold a point at or below a wanted category's bound
      bool any = false;
#pragma unroll
      for (int u = 0; u < BPL; ++u) {
        live[u] &= __ballot((hs[u] && bd[u] <= d2) || (ho[u] && bd[u] <= d3));
        any |= live[u] != 0;
      }
      if (!any) break;
      // the first PER of them in index order; lane l visits point l % kSub of pick l / kSub
      int mine = -1, npick = 0;
#pragma unroll
      for (int s = 0; s < PER; ++s) {
        int pk = -1;
#pragma unroll
        for (int u = 0; u < BPL; ++u)
          if (pk < 0 && live[u]) {
            pk = u * 64 + __ffsll((unsigned long long)live[u]) - 1;
            live[u] &= live[u] - 1;
          }
        if (pk >= 0) ++npick;
        if (lane / kSub == s) mine = pk;
      }
      if (LOAM_ASSOC_PHASE == 0 || LOAM_ASSOC_PHASE == 3) wpts += npick * kSub;
      float ds = 3.4e38f, dot = 3.4e38f;
      const int j = (g + mine) * kSub + lane % kSub;
      if (mine >= 0 && j >= w0 && j < w1 && j != c) {
        const float4 a = L[j];
        const float d = sqdist(a.x, a.y, a.z, sel.x, sel.y, sel.z);
        const uint32_t pos = j > c ? (uint32_t)(j - c - 1) : (1u << 30) + (uint32_t)(c - 1 - j);
        const uint64_t key = ((uint64_t)fkey(d) << 32) | pos;
        if (j >= rs0 && j < rs1) {
          if (want_same) {
            k2 = key < k2 ? key : k2;
            ds = d;
          }
        } else {
          k3 = key < k3 ? key : k3;
          dot = d;
        }
      }
      if (tighten) {
        if (want_same) d2 = fminf(d2, wave_min_f_x(ds));
        d3 = fminf(d3, wave_min_f_x(dot));
      }
    }
  }
  const uint64_t kNone = (uint64_t)fkey(25.0f) << 32;  // keys below this have d < 25 (:491, :602)
  best2 = want_same ? wave_min_u64_x(k2) : ~0ull;
  best3 = wave_min_u64_x(k3);
  if (best2 >= kNone) best2 = ~0ull;
  if (best3 >= kNone) best3 = ~0ull;
}

// a seed's key in wave_window_mono's categories (~0 when j is not in the wanted one or d >= 25)
LOAM_D uint64_t mono_seed_key(const int* rs, int c, int scan, int fwd_end, int j, float d, bool same) {
  if (j < 0 || j == c || !(D(d) < 25)) return ~0ull;
  const int w0 = rs[max(scan - 2, 0)], rs0 = rs[scan], rs1 = rs[scan + 1];
  const int w1 = max(min(fwd_end, rs[min(scan + 3, kRingTab - 1)]), c + 1);
  if (j < w0 || j >= w1 || (j >= rs0 && j < rs1) != same) return ~0ull;
  const uint32_t pos = j > c ? (uint32_t)(j - c - 1) : (1u << 30) + (uint32_t)(c - 1 - j);
  return ((uint64_t)fkey(d) << 32) | pos;
}

LOAM_D int mono_decode(int c, uint64_t k) {
  const uint32_t o = (uint32_t)k;
  return o >= (1u << 30) ? c - 1 - (int)(o - (1u << 30)) : c + 1 + (int)o;
}

// corner association (:478-527): closest (kd NN, sqDis < 25) and the best point of an adjacent
// ring in the index window.  fwd_end = min(cornerPointsSharpNum, C) (Q11).
// A seed (sj, sd): the previous association round's choice for this query and its squared distance
// now (sj < 0: none).  When it belongs to this round's window set (the sets are ring ranges of the
// ring-major Last cloud, see wave_window) it bounds the window minimum, so chunks beyond it are
// skipped; the minimum itself is still taken over every point the walk visits.

// wb: bounds from the nearest neighbour's cells (wave_hash_nn); mono: the cloud is ring-monotone,
// without which no bound is used (window_member would not be exact)
LOAM_D void wave_assoc_corner(const float4* CL, const float4* ch, int fwd_end, uint64_t nn, float4 sel,
                              int sj, int sr, float sd, const WinBound& wb, bool mono, int& ind1, int& ind2,
                              int& wpts, int& wbox) {
  ind1 = -1;
  ind2 = -1;
  if (nn == ~0ull) return;
  const float d0 = __uint_as_float((uint32_t)(nn >> 32));
  if (!(D(d0) < 25)) return;
  const int c = (int)((uint32_t)nn >> 8), scan = (int)((uint32_t)nn & 255u);
  ind1 = c;
  if (LOAM_ASSOC_SKIP & 1) return;
  const float bw = !mono ? 25.0f
                         : fminf(wb.other, sj >= 0 && window_member(sj, sr, c, scan, fwd_end, true, false) ? sd : 25.0f);
  uint64_t best = ~0ull;
  wave_window(CL, ch, c, fwd_end, +1, scan, sel, -1.0f, bw, wpts, wbox, [&](int j, int r, float d) {
    if (r > scan) {
      const uint64_t key = ((uint64_t)fkey(d) << 32) | (uint32_t)(j - c - 1);
      best = key < best ? key : best;
    }
  });
  wave_window(CL, ch, c, fwd_end, -1, scan, sel, -1.0f, bw, wpts, wbox, [&](int j, int r, float d) {
    if (r < scan) {
      const uint64_t key = ((uint64_t)fkey(d) << 32) | (uint32_t)((1u << 30) + (c - 1 - j));
      best = key < best ? key : best;
    }
  });
  best = wave_min_u64_x(best);
  if (best != ~0ull) {
    const uint32_t o = (uint32_t)best;
    ind2 = o >= (1u << 30) ? c - 1 - (int)(o - (1u << 30)) : c + 1 + (int)o;
  }
}

// surface association (:590-650): closest, the best of the same / lower ring (min2) and of the
// higher rings (min3) in the forward window; mirrored in the backward window.
LOAM_D void wave_assoc_surf(const float4* SL, const float4* ch, int fwd_end, uint64_t nn, float4 sel,
                            int sj2, int sr2, float sd2, int sj3, int sr3, float sd3, const WinBound& wb, bool mono,
                            int& ind1, int& ind2, int& ind3, int& wpts, int& wbox) {
  ind1 = ind2 = ind3 = -1;
  if (nn == ~0ull) return;
  const float d0 = __uint_as_float((uint32_t)(nn >> 32));
  if (!(D(d0) < 25)) return;
  const int c = (int)((uint32_t)nn >> 8), scan = (int)((uint32_t)nn & 255u);
  ind1 = c;
  if (LOAM_ASSOC_SKIP & 1) return;
  float b2 = 25.0f, b3 = 25.0f;
  if (mono) {
    b2 = fminf(wb.same, sj2 >= 0 && window_member(sj2, sr2, c, scan, fwd_end, false, true) ? sd2 : 25.0f);
    b3 = fminf(wb.other, sj3 >= 0 && window_member(sj3, sr3, c, scan, fwd_end, false, false) ? sd3 : 25.0f);
  }
  uint64_t best2 = ~0ull, best3 = ~0ull;
  wave_window(SL, ch, c, fwd_end, +1, scan, sel, b2, b3, wpts, wbox, [&](int j, int r, float d) {
    const uint64_t key = ((uint64_t)fkey(d) << 32) | (uint32_t)(j - c - 1);
    if (r <= scan) best2 = key < best2 ? key : best2;
    else best3 = key < best3 ? key : best3;
  });
  wave_window(SL, ch, c, fwd_end, -1, scan, sel, b2, b3, wpts, wbox, [&](int j, int r, float d) {
    const uint64_t key = ((uint64_t)fkey(d) << 32) | (uint32_t)((1u << 30) + (c - 1 - j));
    if (r >= scan) best2 = key < best2 ? key : best2;
    else best3 = key < best3 ? key : best3;
  });
  best2 = wave_min_u64_x(best2);
  best3 = wave_min_u64_x(best3);
  auto decode = [c](uint64_t k) {
    const uint32_t o = (uint32_t)k;
    return o >= (1u << 30) ? c - 1 - (int)(o - (1u << 30)) : c + 1 + (int)o;
  };
  if (best2 != ~0ull) ind2 = decode(best2);
  if (best3 != ~0ull) ind3 = decode(best3);
}

}  // namespace

// ---------------------------------------------------------------- the L-M loop, split per iteration
// Launch sequence per problem batch (od_solve): k_od_begin, then for iter = 0..max_iter-1
// [k_od_assoc when iter % 5 == 0] k_od_rows + k_od_step (fused for small batches), then k_od_fini.
// A problem that has
// converged (or never runs L-M) makes every later launch return at once.

__global__ void k_od_begin(OdBuffers b, FeatView f) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (b.bk_state && blockIdx.x == 0) {  // (one problem: the whole state before this frame touches it)
    for (int k = threadIdx.x; k < kOdStateFloats; k += blockDim.x) b.bk_state[k] = b.state[k];
    for (int k = threadIdx.x; k < kOdStateInts; k += blockDim.x) b.bk_istate[k] = b.istate[k];
    __syncthreads();
  }
  if (p >= b.P) return;
  float* st = b.state + (size_t)p * kOdStateFloats;
  int* ist = b.istate + (size_t)p * kOdStateInts;
  const loampose::Imu imu = load_imu(st);
  const float scanPeriod = 0.1f;  // :461-463 constant-velocity IMU prior (zero without IMU)
  st[3] -= imu.veloX * scanPeriod;
  st[4] -= imu.veloY * scanPeriod;
  st[5] -= imu.veloZ * scanPeriod;
  const int nq = f.count(p, 0) + f.count(p, 2);
  const bool run_lm = ist[kIsCornerLastNum] > 10 && ist[kIsSurfLastNum] > 100;  // :465
  if (run_lm && nq > b.cap_q) ist[kIsErr] |= ERR_CAP_ROWS;
  ist[kIsActive] = (run_lm && nq <= b.cap_q) ? 1 : 0;
  ist[kIsStop] = 0;
  ist[kIsIters] = 0;
  ist[kIsAssoc] = 0;
  ist[kIsRows] = 0;
  ist[kIsDegSteps] = 0;
  ist[kIsNanSkips] = 0;
  ist[kIsGathered] = 0;
  ist[kIsBoxes] = 0;
  b.done[p] = 0;
  if (p == 0 && b.P == 1) ++b.ls_epoch[0];  // (k_od_lm_stream's publication words)
}

// TransformToStart of every query at the current transform (:472, :587), lane per query, for
// the association below (whose waves would otherwise each evaluate it on 64 lanes)
__global__ __launch_bounds__(kOdThreads) void k_od_sel(OdBuffers b, FeatView f) {
  const XcdBlock blk = xcd_block();
  const int p = blk.y;
  const int* ist = b.istate + (size_t)p * kOdStateInts;
  if (!ist[kIsActive] || ist[kIsStop]) return;
  const float* st = b.state + (size_t)p * kOdStateFloats;
  float T[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) T[k] = st[k];
  const int nc = f.count(p, 0), nq = nc + f.count(p, 2);
  const int q = blk.x * kOdThreads + threadIdx.x;
  if (q >= nq) return;
  const float4 po = q < nc ? f.sharp[(size_t)p * f.sharp_stride + q] : f.flat[(size_t)p * f.flat_stride + (q - nc)];
  b.sel[(size_t)p * b.cap_q + q] = loampose::transform_to_start(T, po);
}

// One wave's association queries q0, q0 + G, ... of problem p (:472-527, :587-650): k_od_assoc's
// body, also the association phase of the persistent streaming L-M (k_od_lm_stream).  T: the
// transform for TransformToStart (SEL; otherwise the queries' k_od_sel points are read); seeded:
// ind holds this frame's previous round; cells / bq_*: the wave's LDS scratch (64 entries each);
// rsC / rsS: the Last clouds' ring start tables (LDS); wpts / wbox: the wave's work counters
template <bool SEL>
LOAM_D void od_assoc_wave(const OdBuffers& b, const FeatView& f, int p, int last_buf, int q0, int G, const float* T,
                          bool seeded, int* cells, float4* bq_s4, float4* bq_d, int4* bq_j, const int* rsC,
                          const int* rsS, int& wpts, int& wbox) {
  const int lane = lane_id();
  const int nc = f.count(p, 0), ns = f.count(p, 2), nq = nc + ns;
  const size_t lp = (size_t)last_buf * b.P + p;
  const int C = b.nlast[(p * kOdBufs + last_buf) * 2 + 0], S = b.nlast[(p * kOdBufs + last_buf) * 2 + 1];
  const float4* CL = b.lastC + lp * b.capC;
  const float4* SL = b.lastS + lp * b.capS;
  int* ind = b.ind + (size_t)p * 3 * b.cap_q;
  const bool use_mono = b.P >= b.tune.od_win_mono_min && (b.tune.od_win_mono & (seeded ? 2 : 1)) != 0;
  const bool tight = LOAM_WIN_TIGHTEN == 1 || (LOAM_WIN_TIGHTEN == 2 && !seeded);
  const int hCT = b.hC_T[last_buf * b.P + p], hST = b.hS_T[last_buf * b.P + p];
  const bool monoC = b.mono[lp * 2 + 0] != 0, monoS = b.mono[lp * 2 + 1] != 0;
  // The wave's queries q0, q0 + G, ... in batches of 64: lane l first fetches query l's
  // TransformToStart point and its seeds — the previous round's choices (ind, rounds after the
  // first), their rings and squared distances at this round's transform — for all 64 at once
  // (two dependent loads per batch instead of per query), staged in LDS for the per-query walks.
  for (int i0 = 0; q0 + i0 * G < nq; i0 += 64) {
    {
      const int ql = q0 + (i0 + lane) * G;
      if (ql < nq) {
        float4 s4;
        if constexpr (SEL) {
          const float4 po = ql < nc ? f.sharp[(size_t)p * f.sharp_stride + ql] : f.flat[(size_t)p * f.flat_stride + (ql - nc)];
          s4 = loampose::transform_to_start(T, po);
        } else {
          s4 = b.sel[(size_t)p * b.cap_q + ql];
        }
        const float4* Lc = ql < nc ? CL : SL;
        int j[3] = {-1, -1, -1};
        if (seeded) {
#pragma unroll
          for (int k = 0; k < 3; ++k) j[k] = ind[k * b.cap_q + ql];
        }
        float4 sp[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) sp[k] = j[k] >= 0 ? Lc[j[k]] : make_float4(0, 0, 0, 0);
        const float nnb = j[0] >= 0 ? sqdist(sp[0].x, sp[0].y, sp[0].z, s4.x, s4.y, s4.z) : 3.4e38f;
        const float d1 = sqdist(sp[1].x, sp[1].y, sp[1].z, s4.x, s4.y, s4.z);
        const float d2 = sqdist(sp[2].x, sp[2].y, sp[2].z, s4.x, s4.y, s4.z);
        bq_s4[lane] = s4;
        bq_j[lane] = make_int4(j[0], j[1], j[2], (int)sp[1].w | ((int)sp[2].w << 16));
        bq_d[lane] = make_float4(nnb, d1, d2, 0.0f);
      }
    }
    __builtin_amdgcn_wave_barrier();
    const int nb = min(64, (nq - q0 + G - 1) / G - i0);
    for (int i = 0; i < nb; ++i) {
      const int q = q0 + (i0 + i) * G;
      const float4 s4 = bq_s4[i];
      const int4 jj = bq_j[i];
      const float4 dd = bq_d[i];
      const int j1 = jj.y, j2 = jj.z, r1 = jj.w & 0xffff, r2 = jj.w >> 16;
      const float nnb = dd.x, d1 = dd.y, d2 = dd.z;
      int i1, i2, i3 = -1;
      // the cells' window bounds in the first round only (later rounds have their seeds: the extra
      // pass over the cells cost more than the chunks it saved there)
      WinBound wb;
      if (q < nc && monoC && use_mono) {
        const float4* ch = b.cC + lp * 2 * chunks_of(b.capC);
        const uint64_t nn = wave_hash_nn(b.hC_start + lp * (b.tC + 1), b.hC_pts + lp * b.capC, hCT, CL, ch, C, 1.0f,
                                         1.0f, s4, nnb, cells, wpts, wbox, seeded || !LOAM_WIN_WB ? -1 : 0, min(nc, C), true, &wb);
        i1 = i2 = -1;
        if (nn != ~0ull && D(__uint_as_float((uint32_t)(nn >> 32))) < 25) {
          const int c = (int)((uint32_t)nn >> 8), scan = (int)((uint32_t)nn & 255u), fe = min(nc, C);
          i1 = c;
          uint64_t k2 = ~0ull, k3 = mono_seed_key(rsC, c, scan, fe, j1, d1, false);
          wave_window_mono(CL, b.fC + lp * 2 * subs_of(b.capC), rsC, c, scan, fe, s4, false, wb, tight, k2, k3, wpts, wbox);
          if (k3 != ~0ull) i2 = mono_decode(c, k3);
        }
      } else if (q >= nc && monoS && use_mono) {
        const float4* ch = b.cS + lp * 2 * chunks_of(b.capS);
        const uint64_t nn = wave_hash_nn(b.hS_start + lp * (b.tS + 1), b.hS_pts + lp * b.capS, hST, SL, ch, S, 1.0f,
                                         1.0f, s4, nnb, cells, wpts, wbox, seeded || !LOAM_WIN_WB ? -1 : 1, min(ns, S), true, &wb);
        i1 = i2 = -1;
        if (nn != ~0ull && D(__uint_as_float((uint32_t)(nn >> 32))) < 25) {
          const int c = (int)((uint32_t)nn >> 8), scan = (int)((uint32_t)nn & 255u), fe = min(ns, S);
          i1 = c;
          uint64_t k2 = mono_seed_key(rsS, c, scan, fe, j1, d1, true);
          uint64_t k3 = mono_seed_key(rsS, c, scan, fe, j2, d2, false);
          wave_window_mono(SL, b.fS + lp * 2 * subs_of(b.capS), rsS, c, scan, fe, s4, true, wb, tight, k2, k3, wpts, wbox);
          if (k2 != ~0ull) i2 = mono_decode(c, k2);
          if (k3 != ~0ull) i3 = mono_decode(c, k3);
        }
      } else if (q < nc) {
        const float4* ch = b.cC + lp * 2 * chunks_of(b.capC);
        const uint64_t nn = wave_hash_nn(b.hC_start + lp * (b.tC + 1), b.hC_pts + lp * b.capC, hCT, CL, ch, C, 1.0f,
                                         1.0f, s4, nnb, cells, wpts, wbox, seeded ? -1 : 0, min(nc, C), monoC, &wb);
        wave_assoc_corner(CL, ch, min(nc, C), nn, s4, j1, r1, d1, wb, monoC, i1, i2, wpts, wbox);
      } else {
        const float4* ch = b.cS + lp * 2 * chunks_of(b.capS);
        const uint64_t nn = wave_hash_nn(b.hS_start + lp * (b.tS + 1), b.hS_pts + lp * b.capS, hST, SL, ch, S, 1.0f,
                                         1.0f, s4, nnb, cells, wpts, wbox, seeded ? -1 : 1, min(ns, S), monoS, &wb);
        wave_assoc_surf(SL, ch, min(ns, S), nn, s4, j1, r1, d1, j2, r2, d2, wb, monoS, i1, i2, i3, wpts, wbox);
      }
      if (lane == 0) {
        LOAM_CHECK(q < b.cap_q && p < b.P, q, p);
        LOAM_CHECK(i1 < (q < nc ? C : S) && i2 < (q < nc ? C : S) && i3 < S, i1, i2);
        ind[q] = i1;
        ind[b.cap_q + q] = i2;
        ind[2 * b.cap_q + q] = i3;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// association (:472-527, :587-650), one wave per query: exact NN through the hash, then the
// ring-window scans.
// 8 waves per SIMD (<= 64 VGPRs, <= 100 SGPRs; 7 by default): the association is bound by its
// dependent chain per query, so occupancy is its throughput (measured 3.8 -> 3.2 ms per step)
// COUNT: the profiling variant that also sums the points / chunk boxes it loads into istate
// SEL: the wave computes its query's TransformToStart itself (small batches: one launch fewer per
// association round); otherwise it reads k_od_sel's result
// (measured and removed in round 6: two queries per wave on the wave's halves, round 5: equal or
// slower; per-query certificates that settle a seeded query without a search, round 5: exact, 31 %
// of the queries settled at config 4, but slower: DESIGN.md §15)
template <bool COUNT, bool SEL>
__global__ __launch_bounds__(kAsThreads) __attribute__((amdgpu_waves_per_eu(SEL ? 1 : 8))) void k_od_assoc(OdBuffers b, FeatView f, int last_buf) {
  const XcdBlock blk = xcd_block();
  const int p = blk.y, lane = lane_id(), w = threadIdx.x >> 6;
  const int* ist = b.istate + (size_t)p * kOdStateInts;
  if (!ist[kIsActive] || ist[kIsStop]) return;
  __shared__ int cells[kAsWaves][64];
  __shared__ float4 bq_s4[kAsWaves][64], bq_d[kAsWaves][64];
  __shared__ int4 bq_j[kAsWaves][64];
  __shared__ int rsC[kRingTab], rsS[kRingTab];  // the ring start tables (ring-monotone clouds)
  static_assert(kAsWaves == 1, "the ring tables are loaded by the workgroup's one wave");
  const size_t lp = (size_t)last_buf * b.P + p;
  for (int r = lane; r < kRingTab; r += 64) {
    rsC[r] = b.rstart[lp * 2 * kRingTab + r];
    rsS[r] = b.rstart[lp * 2 * kRingTab + kRingTab + r];
  }
  __builtin_amdgcn_wave_barrier();
  float T[6];
  if constexpr (SEL) {
    const float* st = b.state + (size_t)p * kOdStateFloats;
#pragma unroll
    for (int k = 0; k < 6; ++k) T[k] = st[k];
  }
  int wpts = 0, wbox = 0;  // wave-uniform work counters (loam_stats od_assoc_gathered / _boxes)
  const bool seeded = ist[kIsIters] > 0;  // ind holds this frame's previous round
  od_assoc_wave<SEL>(b, f, p, last_buf, blk.x * kAsWaves + w, gridDim.x * kAsWaves, T, seeded, cells[w], bq_s4[w],
                     bq_d[w], bq_j[w], rsC, rsS, wpts, wbox);
  if (COUNT && lane == 0) {
    if (wpts) atomicAdd((int*)&ist[kIsGathered], wpts);
    if (wbox) atomicAdd((int*)&ist[kIsBoxes], wbox);
  }
}

// the 6x6 step of one iteration (:697-828) of problem p on one lane, from the fixed-order sum of
// the workgroup partials: QR solve / iteration-0 degeneracy analysis, NaN guard, convergence test
// by the whole first wave of the workgroup (jacobi6_wave), the rest on lane 0.  jE / jV: LDS
// for the iteration-0 eigen decomposition
LOAM_D void od_step(const OdBuffers& b, int p, int iter, const double* tot, float* AtA, float* AtB, float* X,
                    float* lm_ws, int* lm_iws, float* jE, float* jV) {
  const int lane = lane_id();
  int* ist = b.istate + (size_t)p * kOdStateInts;
  float* st = b.state + (size_t)p * kOdStateFloats;
  const int nrows = (int)tot[27];
  // lane 0's global reads of the step, issued together up front (each is a round trip on the
  // problem's serial chain): the counters it updates and the transform
  int c_rows = 0, degen = 0, c_deg = 0, c_nan = 0;
  float T[6] = {0, 0, 0, 0, 0, 0};
  if (lane == 0) {
    const int c_assoc = ist[kIsAssoc];
    c_rows = ist[kIsRows];
    degen = ist[kIsDegenerate];
    c_deg = ist[kIsDegSteps];
    c_nan = ist[kIsNanSkips];
#pragma unroll
    for (int q = 0; q < 6; ++q) T[q] = st[q];
    ist[kIsIters] = iter + 1;
    if (iter % 5 == 0) ist[kIsAssoc] = c_assoc + 1;
    ist[kIsRows] = c_rows + nrows;
    if (nrows >= 10) {  // :697-700
      int k = 0;
      for (int i = 0; i < 6; ++i)
        for (int jj = i; jj < 6; ++jj) {
          AtA[i * 6 + jj] = (float)tot[k];
          AtA[jj * 6 + i] = (float)tot[k];
          ++k;
        }
      for (int i = 0; i < 6; ++i) AtB[i] = (float)tot[21 + i];
    }
  }
  if (nrows < 10) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();  // lane 0's AtA / AtB, for the wave
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  bool eig = iter == 0, cert = false;
  if (eig) {
    cert = loamla::nondegenerate_certified(AtA, 10.0f);  // every lane, the same answer
    eig = !cert;
    if (eig) loamla::jacobi6_wave(AtA, jE, jV);
  }
  // the QR solve by the whole wave; lane 0 goes on with X
  loamla::lm_step_wave(AtA, AtB, iter, 10.0f, &degen, st + kOdMatP, X, lm_ws, lm_iws, eig ? jE : nullptr,
                       eig ? jV : nullptr, cert);
  if (lane != 0) return;
  ist[kIsDegenerate] = degen;
  if (degen) ist[kIsDegSteps] = c_deg + 1;
  const bool nan = isnan(X[0]) || isnan(X[1]) || isnan(X[2]) || isnan(X[3]) || isnan(X[4]) || isnan(X[5]);
  if (!nan)  // Q16
    for (int q = 0; q < 6; ++q) st[q] = T[q] + X[q];
  else
    ist[kIsNanSkips] = c_nan + 1;
  const float dR = loamla::delta_r(X), dT = loamla::delta_t(X);
  if (D(dR) < 0.1 && D(dT) < 0.1) ist[kIsStop] = 1;
}

// The residual + weight of a query at this iteration (:530-583 corner, :653-694 surf) from its
// raw point and its associated Last points (t1, t2 and, for a surface query, t3; has: the
// association found them); a rejected correspondence is a zero coefficient (it then adds exact zeros).
LOAM_D void od_coeff_from(int iter, const float* T, float4 po, bool corner, bool has, float4 t1, float4 t2,
                          float4 t3, float4& cf, int& ok) {
  const float4 s4 = loampose::transform_to_start(T, po);
  ok = 0;
  cf = make_float4(0, 0, 0, 0);
  if (corner) {
    if (has) {
      const float x0 = s4.x, y0 = s4.y, z0 = s4.z;
      const float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
      const float m11 = (x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1);
      const float m22 = (x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1);
      const float m33 = (y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1);
      const float a012 = (float)sqrt(D(m11 * m11 + m22 * m22 + m33 * m33));
      const float l12 = (float)sqrt(D((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2)));
      const float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
      const float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
      const float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
      const float ld2 = a012 / l12;
      float sw = 1;
      if (iter >= 5) sw = (float)(1 - 1.8 * fabs(D(ld2)));
      cf = make_float4(sw * la, sw * lb, sw * lc, sw * ld2);
      ok = (D(sw) > 0.1 && ld2 != 0) ? 1 : 0;
    }
  } else if (has) {
    float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
    float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
    float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
    float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
    const float ps = (float)sqrt(D(pa * pa + pb * pb + pc * pc));
    pa /= ps; pb /= ps; pc /= ps; pd /= ps;
    const float pd2 = pa * s4.x + pb * s4.y + pc * s4.z + pd;
    float sw = 1;
    if (iter >= 5)
      sw = (float)(1 - 1.8 * fabs(D(pd2)) / sqrt(sqrt(D(s4.x * s4.x + s4.y * s4.y + s4.z * s4.z))));
    cf = make_float4(sw * pa, sw * pb, sw * pc, sw * pd2);
    ok = (D(sw) > 0.1 && pd2 != 0) ? 1 : 0;
  }
  if (!ok) cf = make_float4(0, 0, 0, 0);
}

// query q's associated Last points (od_coeff_from's t1, t2, t3, has)
LOAM_D bool od_assoc_pts(const OdBuffers& b, int p, int q, int nc, size_t lp, float4& t1, float4& t2, float4& t3) {
  const int* ind = b.ind + (size_t)p * 3 * b.cap_q;
  const int i1 = ind[q], i2 = ind[b.cap_q + q], i3 = ind[2 * b.cap_q + q];
  LOAM_CHECK(q < b.cap_q, q, p);
  LOAM_CHECK(i1 < b.nlast[(p * kOdBufs + (int)(lp / (size_t)b.P)) * 2 + (q < nc ? 0 : 1)], i1, q);
  t1 = t2 = t3 = make_float4(0, 0, 0, 0);
  if (q < nc) {
    if (i2 < 0) return false;
    const float4* CL = b.lastC + lp * b.capC;
    t1 = CL[i1];
    t2 = CL[i2];
    return true;
  }
  if (i2 < 0 || i3 < 0) return false;
  const float4* SL = b.lastS + lp * b.capS;
  t1 = SL[i1];
  t2 = SL[i2];
  t3 = SL[i3];
  return true;
}

// The residual + weight of query q at this iteration against its association
LOAM_D void od_row_coeff(const OdBuffers& b, const FeatView& f, int p, int q, int nc, size_t lp, int iter,
                         const float* T, float4 po, float4& cf, int& ok) {
  LOAM_CHECK(iter < b.max_iter, q, iter);
  float4 t1, t2, t3;
  const bool has = od_assoc_pts(b, p, q, nc, lp, t1, t2, t3);
  od_coeff_from(iter, T, po, q < nc, has, t1, t2, t3, cf, ok);
}

// A stored row was accepted iff its coefficient direction is not zero: od_row_coeff zeroes the
// coefficients of a rejected row, and an accepted row's (x, y, z) is a unit normal times a weight
// above 0.1 (or NaN / inf, which also count), so no separate flag needs to be read back
LOAM_D bool row_ok(const float4& c) { return c.x != 0.0f || c.y != 0.0f || c.z != 0.0f; }

// The coefficient-free factors of each Jacobian entry (:714-753) of a row whose raw point is po:
// every entry is (e0)*coeff.x + (e1)*coeff.y + (e2)*coeff.z with e depending on the raw point and
// the current transform only, evaluated in the reference's expression order
struct OdJf {
  float e00, e01, e02, e10, e12, e20, e21, e22, e30, e31, e32, e40, e41, e42, e50, e51, e52;
};
LOAM_D OdJf od_jfactors(const float* trig, const float* T, float4 po) {
  const float srx = trig[0], crx = trig[1], sry = trig[2], cry = trig[3], srz = trig[4], crz = trig[5];
  const float sw = 1;
  const float tx = sw * T[3], ty = sw * T[4], tz = sw * T[5];
  OdJf e;
  e.e00 = (-sw * crx * sry * srz * po.x + sw * crx * crz * sry * po.y + sw * srx * sry * po.z +
           sw * tx * crx * sry * srz - sw * ty * crx * crz * sry - sw * tz * srx * sry);
  e.e01 = (sw * srx * srz * po.x - sw * crz * srx * po.y + sw * crx * po.z + sw * ty * crz * srx -
           sw * tz * crx - sw * tx * srx * srz);
  e.e02 = (sw * crx * cry * srz * po.x - sw * crx * cry * crz * po.y - sw * cry * srx * po.z +
           sw * tz * cry * srx + sw * ty * crx * cry * crz - sw * tx * crx * cry * srz);
  e.e10 = ((-sw * crz * sry - sw * cry * srx * srz) * po.x + (sw * cry * crz * srx - sw * sry * srz) * po.y -
           sw * crx * cry * po.z + tx * (sw * crz * sry + sw * cry * srx * srz) +
           ty * (sw * sry * srz - sw * cry * crz * srx) + sw * tz * crx * cry);
  e.e12 = ((sw * cry * crz - sw * srx * sry * srz) * po.x + (sw * cry * srz + sw * crz * srx * sry) * po.y -
           sw * crx * sry * po.z + sw * tz * crx * sry - ty * (sw * cry * srz + sw * crz * srx * sry) -
           tx * (sw * cry * crz - sw * srx * sry * srz));
  e.e20 = ((-sw * cry * srz - sw * crz * srx * sry) * po.x + (sw * cry * crz - sw * srx * sry * srz) * po.y +
           tx * (sw * cry * srz + sw * crz * srx * sry) - ty * (sw * cry * crz - sw * srx * sry * srz));
  e.e21 = (-sw * crx * crz * po.x - sw * crx * srz * po.y + sw * ty * crx * srz + sw * tx * crx * crz);
  e.e22 = ((sw * cry * crz * srx - sw * sry * srz) * po.x + (sw * crz * sry + sw * cry * srx * srz) * po.y +
           tx * (sw * sry * srz - sw * cry * crz * srx) - ty * (sw * crz * sry + sw * cry * srx * srz));
  e.e30 = -sw * (cry * crz - srx * sry * srz); e.e31 = sw * crx * srz; e.e32 = sw * (crz * sry + cry * srx * srz);
  e.e40 = -sw * (cry * srz + crz * srx * sry); e.e41 = sw * crx * crz; e.e42 = sw * (sry * srz - cry * crz * srx);
  e.e50 = sw * crx * sry; e.e51 = sw * srx; e.e52 = sw * crx * cry;
  return e;
}

// one row's J (:708-753), B = -0.05 * d2 (:763), JᵀJ / Jᵀb / count added in fp64
LOAM_D void od_row_accum(const OdJf& e, float4 c4, bool okit, double (&acc)[28]) {
  float a[6];
  a[0] = e.e00 * c4.x + e.e01 * c4.y + e.e02 * c4.z;
  a[1] = e.e10 * c4.x + e.e12 * c4.z;
  a[2] = e.e20 * c4.x + e.e21 * c4.y + e.e22 * c4.z;
  a[3] = e.e30 * c4.x + e.e31 * c4.y - e.e32 * c4.z;
  a[4] = e.e40 * c4.x - e.e41 * c4.y - e.e42 * c4.z;
  a[5] = e.e50 * c4.x - e.e51 * c4.y - e.e52 * c4.z;
  const float bb = (float)(-0.05 * D(c4.w));
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int jj = i; jj < 6; ++jj) { acc[k] = loamla::dmac(acc[k], a[i], a[jj]); ++k; }
#pragma unroll
  for (int i = 0; i < 6; ++i) acc[21 + i] = loamla::dmac(acc[21 + i], a[i], bb);
  acc[27] += okit ? 1.0 : 0.0;
}

// Q12 as per-query moments (tuning od_moments_min; NOT bit-identical to the reference, which rounds each
// J entry to float: within the north star's 1e-4).  Every stored row of query q has
// the same raw point (pointOri, :709-712), so at the current transform row r's J is E_q c_r, E_q the
// 6x3 coefficient-free factors (od_jfactors) and c_r the row's (coeff.x, y, z); B_r = -0.05 d2_r.
// Hence the rows' JᵀJ = E_q M_q E_qᵀ and Jᵀb = E_q m_q with M_q = Σ_r c_r c_rᵀ, m_q = Σ_r c_r B_r
// (products of floats, exact in fp64) kept per query across the iterations: O(queries) per
// iteration instead of O(rows), and a rejected row (zero coefficient) still adds nothing.
constexpr int kOdMom = 10;  // Mxx Mxy Mxz Myy Myz Mzz | mx my mz | accepted rows
LOAM_D void od_mom_add(double (&m)[kOdMom], float4 c4) {
  const float bb = (float)(-0.05 * D(c4.w));
  m[0] = loamla::dmac(m[0], c4.x, c4.x);
  m[1] = loamla::dmac(m[1], c4.x, c4.y);
  m[2] = loamla::dmac(m[2], c4.x, c4.z);
  m[3] = loamla::dmac(m[3], c4.y, c4.y);
  m[4] = loamla::dmac(m[4], c4.y, c4.z);
  m[5] = loamla::dmac(m[5], c4.z, c4.z);
  m[6] = loamla::dmac(m[6], c4.x, bb);
  m[7] = loamla::dmac(m[7], c4.y, bb);
  m[8] = loamla::dmac(m[8], c4.z, bb);
  m[9] += row_ok(c4) ? 1.0 : 0.0;
}
// the query's JᵀJ (21) | Jᵀb (6) | rows (1) from its moments at the current factors e, added to acc
LOAM_D void od_mom_accum(const OdJf& e, const double (&m)[kOdMom], double (&acc)[28]) {
  // E rows in od_row_accum's signs (a[1] has no y term)
  const double E[6][3] = {{e.e00, e.e01, e.e02}, {e.e10, 0.0, e.e12},   {e.e20, e.e21, e.e22},
                          {e.e30, e.e31, -e.e32}, {e.e40, -e.e41, -e.e42}, {e.e50, -e.e51, -e.e52}};
  // (no rounding order to match here: fused multiply-adds throughout)
  auto dot3 = [](double a0, double a1, double a2, double b0, double b1, double b2) {
    return __builtin_fma(a0, b0, __builtin_fma(a1, b1, a2 * b2));
  };
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    // F = E_i M (M symmetric)
    const double f0 = dot3(E[i][0], E[i][1], E[i][2], m[0], m[1], m[2]);
    const double f1 = dot3(E[i][0], E[i][1], E[i][2], m[1], m[3], m[4]);
    const double f2 = dot3(E[i][0], E[i][1], E[i][2], m[2], m[4], m[5]);
#pragma unroll
    for (int jj = i; jj < 6; ++jj) { acc[k] += dot3(f0, f1, f2, E[jj][0], E[jj][1], E[jj][2]); ++k; }
    acc[21 + i] += dot3(E[i][0], E[i][1], E[i][2], m[6], m[7], m[8]);
  }
  acc[27] += m[9];
}


// one iteration's rows (lane per query): this iteration's residual + weight stored at [iter][q];
// then the Jacobian of every row accumulated so far (Q12: rows of iterations 0..iter, all
// evaluated at the current transform, :708-764) summed in fp64 into this workgroup's partial
// JᵀJ / Jᵀb / row count; k_od_step sums the partials.  Large batches.
// FUSED: the last workgroup of the problem to finish sums the gq partials (in k_od_step's order)
// and runs the step itself, instead of a k_od_step launch per iteration.
constexpr int kOdRowsWpe = 4;  // <= 128 VGPRs with two rows' loads in flight
// INF: stored rows whose loads are in flight together per lane step (2, the one instantiation: 8 for
// small batches, tuning od_rows_deep_max until round 6, measured no faster and was removed)
// MOM: the stored rows as the query's fp64 moments (od_mom_add / od_mom_accum; tuning od_moments_min)
// instead of re-evaluating each (INF unused)
template <bool FUSED, int INF, bool MOM = false>
__global__ __launch_bounds__(kOdThreads) __attribute__((amdgpu_waves_per_eu(INF > 2 ? 2 : kOdRowsWpe))) void k_od_rows(OdBuffers b, FeatView f, int last_buf, int iter) {
  const XcdBlock blk = xcd_block();
  const int p = blk.y, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int* ist = b.istate + (size_t)p * kOdStateInts;
  if (!ist[kIsActive] || ist[kIsStop]) return;
  __shared__ double red[kOdWaves][28];
  __shared__ float trig[6];
  const float* st = b.state + (size_t)p * kOdStateFloats;
  float T[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) T[k] = st[k];
  if (tid < 6) {  // the angles' double sin / cos as floats, one per lane (trig[2k], trig[2k + 1]: sin, cos of T[k])
    const float ang = st[tid >> 1];
    trig[tid] = (float)((tid & 1) ? dcos(ang) : dsin(ang));
  }
  const int nc = f.count(p, 0), ns = f.count(p, 2), nq = nc + ns;
  const int q = blk.x * kOdThreads + tid;
  const size_t lp = (size_t)last_buf * b.P + p;
  float4* qcf = b.q_cf + (size_t)p * b.max_iter * b.cap_q;
  int8_t* qok = b.q_ok + (size_t)p * b.max_iter * b.cap_q;
  float4 po = make_float4(0, 0, 0, 0);
  double acc[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) acc[k] = 0.0;
  if constexpr (MOM) {
    double m[kOdMom];
    if (q < nq) {
      po = q < nc ? f.sharp[(size_t)p * f.sharp_stride + q] : f.flat[(size_t)p * f.flat_stride + (q - nc)];
      float4 cf;
      int ok;
      od_row_coeff(b, f, p, q, nc, lp, iter, T, po, cf, ok);
      double* mq = b.mom + (size_t)p * kOdMom * b.cap_q + q;  // [P][kOdMom][cap_q]
#pragma unroll
      for (int k = 0; k < kOdMom; ++k) m[k] = iter == 0 ? 0.0 : mq[(size_t)k * b.cap_q];
      od_mom_add(m, cf);
#pragma unroll
      for (int k = 0; k < kOdMom; ++k) mq[(size_t)k * b.cap_q] = m[k];
    }
    __syncthreads();  // trig
    if (q < nq) od_mom_accum(od_jfactors(trig, T, po), m, acc);
  } else {
  if (q < nq) {
    po = q < nc ? f.sharp[(size_t)p * f.sharp_stride + q] : f.flat[(size_t)p * f.flat_stride + (q - nc)];
    float4 cf;
    int ok;
    od_row_coeff(b, f, p, q, nc, lp, iter, T, po, cf, ok);
    qcf[(size_t)iter * b.cap_q + q] = cf;
    qok[(size_t)iter * b.cap_q + q] = (int8_t)ok;
  }
  __syncthreads();
  if (q < nq) {
    const OdJf e = od_jfactors(trig, T, po);
    // the stored rows INF iterations at a time (their loads in flight together), summed in order
    for (int it0 = 0; it0 <= iter; it0 += INF) {
      float4 cv4[INF];
      bool okv[INF];
#pragma unroll
      for (int u = 0; u < INF; ++u) {
        const int it = it0 + u;
        cv4[u] = it <= iter ? qcf[(size_t)it * b.cap_q + q] : make_float4(0, 0, 0, 0);
        okv[u] = row_ok(cv4[u]);
      }
#pragma unroll
      for (int u = 0; u < INF; ++u)
        if (it0 + u <= iter) od_row_accum(e, cv4[u], okv[u], acc);
    }
  }
  }
  // wave sums of the 28 values as a butterfly reduce-scatter (32 shuffles instead of 28 x 6);
  // lanes 2v, 2v+1 end with the sum of value v
  wave_reduce_scatter_28(acc);
  if ((lane & 1) == 0 && (lane >> 1) < 28) red[w][lane >> 1] = acc[0];
  __syncthreads();
  if (tid < 28) {
    double v = red[0][tid];
    for (int ww = 1; ww < kOdWaves; ++ww) v += red[ww][tid];
    if (FUSED) store_partial(&b.part[((size_t)p * b.gq + blk.x) * 28 + tid], v);
    else b.part[((size_t)p * b.gq + blk.x) * 28 + tid] = v;
  }
  if constexpr (FUSED) {
    __shared__ int sh_last;
    __shared__ double tot[28];
    __shared__ float AtA[36], AtB[6], X[6], lm_ws[loamla::kLmWs], jE[6], jV[36];
    __shared__ int lm_iws[12];
    __syncthreads();
    // (store_partial / arrive_last: write-through partials, relaxed counter; the last workgroup
    // acquires at agent scope, then reads them with sc1 loads)
    if (tid == 0) sh_last = arrive_last(&b.done[p], b.gq);
    __syncthreads();
    if (!sh_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (tid < 28) {  // k_od_step's fixed order over the workgroups; eight partials in flight per step
      double v = 0.0;
      const double* pp = b.part + (size_t)p * b.gq * 28 + tid;
      for (int g = 0; g < b.gq; g += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          t[u] = g + u < b.gq ? __hip_atomic_load(&pp[(size_t)(g + u) * 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (g + u < b.gq) v += t[u];
      }
      tot[tid] = v;
    }
    __syncthreads();
    if (tid < 64) {  // the first wave
      if (tid == 0) b.done[p] = 0;
      od_step(b, p, iter, tot, AtA, AtB, X, lm_ws, lm_iws, jE, jV);
    }
  }
}

// The rows launch of the per-query moments (tuning od_moments_min; k_od_rows<., ., true>'s sums)
// shaped for latency: a launch is a few dependent global round trips per lane, so the independent
// loads (the problem's flags, transform and counts, the query's moments and round data) are issued
// together ahead of the early return, and a query's associated Last points are gathered through ind
// only in the first iteration of an association round (Q10), which keeps them in b.qa for the
// round's other four (one round trip instead of two).  Sums in k_od_rows' order: the same bits.
template <bool FUSED>
__global__ __launch_bounds__(kOdThreads) __attribute__((amdgpu_waves_per_eu(kOdRowsWpe))) void k_od_rows_mom(OdBuffers b, FeatView f, int last_buf, int iter) {
  const XcdBlock blk = xcd_block();
  const int p = blk.y, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int* ist = b.istate + (size_t)p * kOdStateInts;
  const float* st = b.state + (size_t)p * kOdStateFloats;
  const int q = blk.x * kOdThreads + tid;
  const bool inq = q < b.cap_q, first = iter % 5 == 0;
  // round trip 1: everything that depends on q and p only
  const int active = ist[kIsActive], stop = ist[kIsStop];
  const int nc = f.count(p, 0), ns = f.count(p, 2);
  float T[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) T[k] = st[k];
  double* mq = b.mom + (size_t)p * kOdMom * b.cap_q + q;  // [P][kOdMom][cap_q]
  float4* qa = b.qa + ((size_t)p * b.cap_q + q) * 3;     // [P][cap_q][3]
  double m[kOdMom];
#pragma unroll
  for (int k = 0; k < kOdMom; ++k) m[k] = iter > 0 && inq ? mq[(size_t)k * b.cap_q] : 0.0;
  float4 t1 = make_float4(0, 0, 0, 0), t2 = t1, t3 = t1;
  int i1 = -1, i2 = -1, i3 = -1;
  if (inq) {
    if (first) {
      const int* ind = b.ind + (size_t)p * 3 * b.cap_q;
      i1 = ind[q];
      i2 = ind[b.cap_q + q];
      i3 = ind[2 * b.cap_q + q];
    } else {
      t1 = qa[0];
      t2 = qa[1];
      t3 = qa[2];
    }
  }
  if (!active || stop) return;
  __shared__ double red[kOdWaves][28];
  __shared__ float trig[6];
  if (tid < 6) {  // the angles' double sin / cos as floats, one per lane (trig[2k], trig[2k + 1]: sin, cos of T[k])
    const float ang = T[tid >> 1];
    trig[tid] = (float)((tid & 1) ? dcos(ang) : dsin(ang));
  }
  const int nq = nc + ns;
  float4 po = make_float4(0, 0, 0, 0);
  double acc[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) acc[k] = 0.0;
  if (q < nq) {
    // round trip 2: the raw point (its cloud by nc) and, in a round's first iteration, the points
    po = q < nc ? f.sharp[(size_t)p * f.sharp_stride + q] : f.flat[(size_t)p * f.flat_stride + (q - nc)];
    if (first) {  // od_assoc_pts; t1.w: the association holds
      const size_t lp = (size_t)last_buf * b.P + p;
      bool has;
      if (q < nc) {
        has = i2 >= 0;
        if (has) {
          const float4* CL = b.lastC + lp * b.capC;
          t1 = CL[i1];
          t2 = CL[i2];
        }
      } else {
        has = i2 >= 0 && i3 >= 0;
        if (has) {
          const float4* SL = b.lastS + lp * b.capS;
          t1 = SL[i1];
          t2 = SL[i2];
          t3 = SL[i3];
        }
      }
      t1.w = has ? 1.0f : 0.0f;
      qa[0] = t1;
      qa[1] = t2;
      qa[2] = t3;
    }
    float4 cf;
    int ok;
    od_coeff_from(iter, T, po, q < nc, t1.w != 0.0f, t1, t2, t3, cf, ok);
    od_mom_add(m, cf);
#pragma unroll
    for (int k = 0; k < kOdMom; ++k) mq[(size_t)k * b.cap_q] = m[k];
  }
  __syncthreads();  // trig
  if (q < nq) od_mom_accum(od_jfactors(trig, T, po), m, acc);
  wave_reduce_scatter_28(acc);
  if ((lane & 1) == 0 && (lane >> 1) < 28) red[w][lane >> 1] = acc[0];
  __syncthreads();
  if (tid < 28) {
    double v = red[0][tid];
    for (int ww = 1; ww < kOdWaves; ++ww) v += red[ww][tid];
    if (FUSED) store_partial(&b.part[((size_t)p * b.gq + blk.x) * 28 + tid], v);
    else b.part[((size_t)p * b.gq + blk.x) * 28 + tid] = v;
  }
  if constexpr (FUSED) {
    __shared__ int sh_last;
    __shared__ double tot[28];
    __shared__ float AtA[36], AtB[6], X[6], lm_ws[loamla::kLmWs], jE[6], jV[36];
    __shared__ int lm_iws[12];
    __syncthreads();
    if (tid == 0) sh_last = arrive_last(&b.done[p], b.gq);
    __syncthreads();
    if (!sh_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (tid < 28) {  // k_od_step's fixed order over the workgroups; eight partials in flight per step
      double v = 0.0;
      const double* pp = b.part + (size_t)p * b.gq * 28 + tid;
      for (int g = 0; g < b.gq; g += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          t[u] = g + u < b.gq ? __hip_atomic_load(&pp[(size_t)(g + u) * 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (g + u < b.gq) v += t[u];
      }
      tot[tid] = v;
    }
    __syncthreads();
    if (tid < 64) {  // the first wave
      if (tid == 0) b.done[p] = 0;
      od_step(b, p, iter, tot, AtA, AtB, X, lm_ws, lm_iws, jE, jV);
    }
  }
}

// Small batches (streaming, config 2): a workgroup per (256 queries, stored iteration) pair, each
// lane one row, so the Q12 re-evaluation of every stored row is one load deep instead of a chain
// of (iter + 1) per lane; the workgroups of the current iteration compute and store the new
// residuals.  The last workgroup of the problem to finish sums the gq * (iter + 1) partials in a
// fixed order and runs the 6x6 step (one launch per iteration).
__global__ __launch_bounds__(kOdThreads) void k_od_rows_small(OdBuffers b, FeatView f, int last_buf, int iter) {
  const int p = blockIdx.y, it = blockIdx.z, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int* ist = b.istate + (size_t)p * kOdStateInts;
  if (!ist[kIsActive] || ist[kIsStop]) return;
  LOAM_PH(const unsigned long long ph0 = ph_now(); if (tid == 0) ph_start(&g_ph_od, ph0);)
  __shared__ double red[kOdWaves][28];
  __shared__ float trig[6];
  const float* st = b.state + (size_t)p * kOdStateFloats;
  float T[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) T[k] = st[k];
  if (tid < 6) {  // the angles' double sin / cos as floats, one per lane (trig[2k], trig[2k + 1]: sin, cos of T[k])
    const float ang = st[tid >> 1];
    trig[tid] = (float)((tid & 1) ? dcos(ang) : dsin(ang));
  }
  const int nc = f.count(p, 0), ns = f.count(p, 2), nq = nc + ns;
  const int q = blockIdx.x * kOdThreads + tid;
  const size_t lp = (size_t)last_buf * b.P + p;
  float4* qcf = b.q_cf + (size_t)p * b.max_iter * b.cap_q;
  int8_t* qok = b.q_ok + (size_t)p * b.max_iter * b.cap_q;
  float4 po = make_float4(0, 0, 0, 0), c4 = po;
  bool okit = false;
  if (q < nq) {
    po = q < nc ? f.sharp[(size_t)p * f.sharp_stride + q] : f.flat[(size_t)p * f.flat_stride + (q - nc)];
    if (it == iter) {
      int ok;
      od_row_coeff(b, f, p, q, nc, lp, iter, T, po, c4, ok);
      okit = ok != 0;
      qcf[(size_t)iter * b.cap_q + q] = c4;
      qok[(size_t)iter * b.cap_q + q] = (int8_t)ok;
    } else {
      c4 = qcf[(size_t)it * b.cap_q + q];
      okit = row_ok(c4);
    }
  }
  __syncthreads();
  double acc[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) acc[k] = 0.0;
  if (q < nq) od_row_accum(od_jfactors(trig, T, po), c4, okit, acc);
  wave_reduce_scatter_28(acc);
  if ((lane & 1) == 0 && (lane >> 1) < 28) red[w][lane >> 1] = acc[0];
  __syncthreads();
  const int G = (int)gridDim.x * (iter + 1), g = it * (int)gridDim.x + (int)blockIdx.x;
  if (tid < 28) {
    double v = red[0][tid];
    for (int ww = 1; ww < kOdWaves; ++ww) v += red[ww][tid];
    store_partial(&b.part[((size_t)p * b.gq * b.max_iter + g) * 28 + tid], v);
  }
  __shared__ int sh_last;
  __shared__ double tot[28];
  __shared__ float AtA[36], AtB[6], X[6], lm_ws[loamla::kLmWs], jE[6], jV[36];
  __shared__ int lm_iws[12];
  __syncthreads();
  LOAM_PH(const int phk = iter == 0 ? 0 : 1; const unsigned long long ph1 = ph_now();
          if (tid == 0) ph_arrive(&g_ph_od, phk, ph0, ph1);)
  // (store_partial / arrive_last: the partials are drained write-through before the counter add;
  // the last workgroup acquires at agent scope, then reads them with sc1 loads)
  if (tid == 0)
    sh_last = arrive_last(&b.done[p], G);
  __syncthreads();
  if (!sh_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  LOAM_PH(const unsigned long long ph2 = ph_now();)
  // fixed-order sum of the G partials: thread (slice s, value v) sums partials s, s + 8, ... with
  // all its loads in flight at once, then the eight slice sums are added in slice order
  __shared__ double slice[8][28];
  if (tid < 8 * 28) {
    const int v = tid % 28, sl = tid / 28;
    const double* pp = b.part + (size_t)p * b.gq * b.max_iter * 28 + v;
    // the slice's partials in order, sixteen loads in flight per round (G grows to gq * (iter + 1))
    double acc1 = 0.0;
    for (int g0 = sl; g0 < G; g0 += 8 * 16) {
      double t16[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int g = g0 + 8 * u;
        t16[u] = g < G ? __hip_atomic_load(&pp[(size_t)g * 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (g0 + 8 * u < G) acc1 += t16[u];
    }
    slice[sl][v] = acc1;
  }
  __syncthreads();
  if (tid < 28) {
    double v = slice[0][tid];
#pragma unroll
    for (int sl = 1; sl < 8; ++sl) v += slice[sl][tid];
    tot[tid] = v;
  }
  __syncthreads();
  LOAM_PH(const unsigned long long ph3 = ph_now();)
  if (tid < 64) {  // the first wave
    if (tid == 0) b.done[p] = 0;
    od_step(b, p, iter, tot, AtA, AtB, X, lm_ws, lm_iws, jE, jV);
    LOAM_PH(const unsigned long long ph4 = ph_now(); if (tid == 0) ph_last(&g_ph_od, phk, ph1, ph2, ph3, ph4);)
  }
}

// ---- the one-problem L-M as one persistent launch (streaming: the config-3 chain, config 2) ----
// The launch-per-iteration form pays a dispatch and a grid-wide hand-off per iteration (25 rows
// launches + 5 association launches per sweep, ~8 us each plus the gaps between them).  Here G
// workgroups of kOdLsThreads stay resident for the whole loop.  Each query belongs to one wave
// for the association and to its workgroup for the rows (its stored coefficients of earlier
// iterations, Q12, are read back only by the workgroup that wrote them), so the one exchange per
// iteration is the 28 partial sums: every workgroup publishes its partial with write-through
// stores and a publication word, reads all G partials, sums them in workgroup order and runs the
// step itself — the same sums and the same code in every workgroup, so every workgroup holds the
// same transform and takes the same convergence decision, with no second hand-off.  Partials are
// double-buffered by iteration parity (a workgroup can be at most one iteration ahead of the
// slowest).  Co-residency of the G workgroups is checked on the host (od_solve); a workgroup
// waits only for partials of the current iteration, which every resident workgroup produces.
constexpr int kOdLsThreads = 512, kOdLsWaves = kOdLsThreads / 64;

// the workgroup-local L-M state (LDS): od_step's global state for the persistent kernel
struct OdLsState {
  float T[6], matP[36], trig[6];
  int degen, iters, assoc, rows, deg_steps, nan_skips, stop;
};

// od_step on the workgroup-local state (wave 0): the same reads, arithmetic and decisions
LOAM_D void od_step_ls(int iter, const double* tot, OdLsState& S, float* AtA, float* AtB, float* X, float* lm_ws,
                       int* lm_iws, float* jE, float* jV) {
  const int lane = lane_id();
  const int nrows = (int)tot[27];
  if (lane == 0) {
    S.iters = iter + 1;
    if (iter % 5 == 0) ++S.assoc;
    S.rows += nrows;
    if (nrows >= 10) {  // :697-700
      int k = 0;
      for (int i = 0; i < 6; ++i)
        for (int jj = i; jj < 6; ++jj) {
          AtA[i * 6 + jj] = (float)tot[k];
          AtA[jj * 6 + i] = (float)tot[k];
          ++k;
        }
      for (int i = 0; i < 6; ++i) AtB[i] = (float)tot[21 + i];
    }
  }
  if (nrows < 10) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  bool eig = iter == 0, cert = false;
  if (eig) {
    cert = loamla::nondegenerate_certified(AtA, 10.0f);
    eig = !cert;
    if (eig) loamla::jacobi6_wave(AtA, jE, jV);
  }
  int degen = S.degen;
  loamla::lm_step_wave(AtA, AtB, iter, 10.0f, &degen, S.matP, X, lm_ws, lm_iws, eig ? jE : nullptr, eig ? jV : nullptr,
                       cert);
  if (lane != 0) return;
  S.degen = degen;
  if (degen) ++S.deg_steps;
  const bool nan = isnan(X[0]) || isnan(X[1]) || isnan(X[2]) || isnan(X[3]) || isnan(X[4]) || isnan(X[5]);
  if (!nan)  // Q16
    for (int q = 0; q < 6; ++q) S.T[q] = S.T[q] + X[q];
  else
    ++S.nan_skips;
  const float dR = loamla::delta_r(X), dT = loamla::delta_t(X);
  if (D(dR) < 0.1 && D(dT) < 0.1) S.stop = 1;
}

__global__ __launch_bounds__(kOdLsThreads) void k_od_lm_stream(OdBuffers b, FeatView f, int last_buf) {
  constexpr int NW = kOdLsWaves;
  const int g = blockIdx.x, G = gridDim.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6, p = 0;
  int* ist = b.istate;
  float* st = b.state;
  if (!ist[kIsActive] || ist[kIsStop]) return;  // (the same value in every workgroup)
  __shared__ int cells[NW][64];
  __shared__ float4 bq_s4[NW][64], bq_d[NW][64];
  __shared__ int4 bq_j[NW][64];
  __shared__ int rsC[kRingTab], rsS[kRingTab];
  __shared__ double red[NW][28], slice[8][28], tot[28];
  __shared__ float AtA[36], AtB[6], X[6], lm_ws[loamla::kLmWs], jE[6], jV[36];
  __shared__ int lm_iws[12];
  __shared__ OdLsState S;
  __shared__ unsigned long long sh_epoch;
  const size_t lp = (size_t)last_buf * b.P + p;
  for (int r = tid; r < kRingTab; r += kOdLsThreads) {
    rsC[r] = b.rstart[lp * 2 * kRingTab + r];
    rsS[r] = b.rstart[lp * 2 * kRingTab + kRingTab + r];
  }
  if (tid < 6) S.T[tid] = st[tid];
  if (tid < 36) S.matP[tid] = st[kOdMatP + tid];
  if (tid == 0) {
    S.degen = ist[kIsDegenerate];
    S.iters = 0;
    S.assoc = 0;
    S.rows = 0;
    S.deg_steps = 0;
    S.nan_skips = 0;
    S.stop = 0;
    sh_epoch = b.ls_epoch[0];
  }
  __syncthreads();
  if (tid < 6) S.trig[tid] = (float)((tid & 1) ? dcos(S.T[tid >> 1]) : dsin(S.T[tid >> 1]));
  const int nc = f.count(p, 0), ns = f.count(p, 2), nq = nc + ns;
  const int Wt = G * NW;                 // association waves: wave (g, w) takes queries g NW + w + k Wt
  const int nloc = nq > g * NW ? ((nq - g * NW - 1) / Wt + 1) * NW : 0;  // (an upper bound; q < nq tested)
  float4* qcf = b.q_cf;
  const unsigned long long tag0 = sh_epoch << 16;  // (iterations + 1 <= 1001 < 2^16: loam_create bounds max_iter)
  int wpts = 0, wbox = 0;
  __syncthreads();
  for (int it = 0; it < b.max_iter; ++it) {
    if (it % 5 == 0) {  // Q10
      float T[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) T[k] = S.T[k];
      od_assoc_wave<true>(b, f, p, last_buf, g * NW + w, Wt, T, it > 0, cells[w], bq_s4[w], bq_d[w], bq_j[w], rsC, rsS,
                          wpts, wbox);
      __syncthreads();  // (the rows below read the association of this workgroup's queries)
    }
    // rows: every (query of this workgroup, stored iteration) pair re-evaluated at the current
    // transform; the current iteration's coefficient computed and stored first by its own pair
    double acc[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) acc[k] = 0.0;
    {
      float T[6], trig[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) { T[k] = S.T[k]; trig[k] = S.trig[k]; }
      const int npair = nloc * (it + 1);
      for (int e = tid; e < npair; e += kOdLsThreads) {
        const int l = e % nloc, its = e / nloc;
        const int q = g * NW + (l % NW) + (l / NW) * Wt;
        if (q >= nq) continue;
        const float4 po = q < nc ? f.sharp[(size_t)p * f.sharp_stride + q] : f.flat[(size_t)p * f.flat_stride + (q - nc)];
        float4 c4;
        bool okit;
        if (its == it) {
          int ok;
          od_row_coeff(b, f, p, q, nc, lp, it, T, po, c4, ok);
          okit = ok != 0;
          qcf[(size_t)it * b.cap_q + q] = c4;
        } else {
          c4 = qcf[(size_t)its * b.cap_q + q];
          okit = row_ok(c4);
        }
        od_row_accum(od_jfactors(trig, T, po), c4, okit, acc);
      }
    }
    wave_reduce_scatter_28(acc);
    if ((lane & 1) == 0 && (lane >> 1) < 28) red[w][lane >> 1] = acc[0];
    __syncthreads();
    const int par = it & 1;
    if (tid < 28) {  // this workgroup's partial, waves in order, stored write-through
      double v = red[0][tid];
      for (int ww = 1; ww < NW; ++ww) v += red[ww][tid];
      store_partial(&b.ls_part[((size_t)par * kOdLsMaxG + g) * 28 + tid], v);
    }
    if (tid < 64) {
      __builtin_amdgcn_wave_barrier();  // (every lane's store drained: store_partial waits for it)
      if (tid == 0)
        __hip_atomic_store(&b.ls_flag[g], tag0 + (unsigned long long)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every workgroup's partial of this iteration
    if (tid < G) {
      const unsigned long long want = tag0 + (unsigned long long)(it + 1);
      while (__hip_atomic_load(&b.ls_flag[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want)
        __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
    if (tid < 8 * 28) {  // fixed order: slice s sums partials s, s + 8, ...; the slices in order
      const int v = tid % 28, sl = tid / 28;
      const double* pp = b.ls_part + (size_t)par * kOdLsMaxG * 28 + v;
      double a = 0.0;
      for (int g0 = sl; g0 < G; g0 += 8 * 8) {
        double t8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int gg = g0 + 8 * u;
          t8[u] = gg < G ? __hip_atomic_load(&pp[(size_t)gg * 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (g0 + 8 * u < G) a += t8[u];
      }
      slice[sl][v] = a;
    }
    __syncthreads();
    if (tid < 28) {
      double v = slice[0][tid];
#pragma unroll
      for (int sl = 1; sl < 8; ++sl) v += slice[sl][tid];
      tot[tid] = v;
    }
    __syncthreads();
    if (tid < 64) od_step_ls(it, tot, S, AtA, AtB, X, lm_ws, lm_iws, jE, jV);
    __syncthreads();
    if (S.stop) break;
    if (tid < 6) S.trig[tid] = (float)((tid & 1) ? dcos(S.T[tid >> 1]) : dsin(S.T[tid >> 1]));
    __syncthreads();
  }
  if (g == 0) {  // the state for the kernels after the loop (the same in every workgroup)
    if (tid < 6) st[tid] = S.T[tid];
    if (tid < 36) st[kOdMatP + tid] = S.matP[tid];
    if (tid == 0) {
      ist[kIsDegenerate] = S.degen;
      ist[kIsIters] = S.iters;
      ist[kIsAssoc] = S.assoc;
      ist[kIsRows] = S.rows;
      ist[kIsDegSteps] = S.deg_steps;
      ist[kIsNanSkips] = S.nan_skips;
      ist[kIsStop] = S.stop;
    }
  }
  if (lane == 0) {  // (work counters: every wave's association)
    if (wpts) atomicAdd((int*)&ist[kIsGathered], wpts);
    if (wbox) atomicAdd((int*)&ist[kIsBoxes], wbox);
  }
}

// workgroups of k_od_lm_stream for a query capacity (one association wave per query up to
// kOdLsMaxG workgroups), or 0 when they could not all be resident at once (the per-iteration
// launches run instead)
int od_lm_stream_grid(int cap_q) {
  static int cap[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_od_lm_stream, kOdLsThreads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      per_cu = cus = 0;
    cap[dev] = std::max(1, per_cu * cus);
  }
  const int G = std::min(kOdLsMaxG, (cap_q + kOdLsWaves - 1) / kOdLsWaves);
  return 2 * G <= cap[dev] ? G : 0;  // (a margin of 2: other streams' kernels may hold slots a while)
}

// the step as its own launch (large batches): one wave per problem
__global__ __launch_bounds__(64) void k_od_step(OdBuffers b, int iter, int gq) {
  const int p = blockIdx.x, lane = threadIdx.x;
  const int* ist = b.istate + (size_t)p * kOdStateInts;
  if (!ist[kIsActive] || ist[kIsStop]) return;
  __shared__ double tot[28];
  __shared__ float AtA[36], AtB[6], X[6], lm_ws[loamla::kLmWs], jE[6], jV[36];
  __shared__ int lm_iws[12];
  if (lane < 28) {  // fixed order over the workgroups; eight partials in flight per step
    double v = 0.0;
    const double* pp = b.part + (size_t)p * b.gq * 28 + lane;
    for (int g = 0; g < gq; g += 8) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = g + u < gq ? pp[(size_t)(g + u) * 28] : 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (g + u < gq) v += t[u];
    }
    tot[lane] = v;
  }
  __syncthreads();
  od_step(b, p, iter, tot, AtA, AtB, X, lm_ws, lm_iws, jE, jV);
}

// pose accumulation (:830-856) for every problem
__global__ __launch_bounds__(64) void k_od_fini(OdBuffers b, FeatView f) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= b.P) return;
  float* st = b.state + (size_t)p * kOdStateFloats;
  int* ist = b.istate + (size_t)p * kOdStateInts;
  const loampose::Imu imu = load_imu(st);
  loampose::accumulate_pose(st, imu, st + kOdSum);
  ist[kIsQueries] = ist[kIsAssoc] * (f.count(p, 0) + f.count(p, 2));
}

// TransformToEnd of lessSharp / lessFlat (and full) into Last[dst] / fullEnd[dst] (:875-891).
// mode 0: copy raw (the init frame, :427-434); 1: zero transform (batch seeding); 2: solved transform
__global__ __launch_bounds__(256) void k_od_end(OdBuffers b, FeatView f, int dst, int mode, int do_full) {
  const int p = blockIdx.y;
  const float* st = b.state + (size_t)p * kOdStateFloats;
  float t[6] = {0, 0, 0, 0, 0, 0};
  loampose::Imu imu = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (mode == 2) {
    for (int k = 0; k < 6; ++k) t[k] = st[k];
    imu = load_imu(st);
  }
  const int nl = f.count(p, 1), nf = f.count(p, 3), nfull = do_full ? f.nfull(p) : 0;
  const int cl = min(nl, b.capC), cf = min(nf, b.capS), cu = min(nfull, b.capS);
  const int total = cl + cf + cu;
  float4* oc = b.lastC + ((size_t)dst * b.P + p) * b.capC;
  float4* os = b.lastS + ((size_t)dst * b.P + p) * b.capS;
  float4* ofl = b.fullEnd + ((size_t)dst * b.P + p) * b.capS;
  const loampose::EndRot er = loampose::end_rot_wave(t, imu);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    float4 a;
    float4* o;
    if (i < cl) { a = f.lsharp[(size_t)p * f.lsharp_stride + i]; o = oc + i; }
    else if (i < cl + cf) { a = f.lflat[(size_t)p * f.lflat_stride + (i - cl)]; o = os + (i - cl); }
    else { a = f.full[(size_t)p * f.full_stride + (i - cl - cf)]; o = ofl + (i - cl - cf); }
    *o = mode == 0 ? a : loampose::transform_to_end(t, imu, er, a, mode == 1);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    b.nlast[(p * kOdBufs + dst) * 2 + 0] = cl;
    b.nlast[(p * kOdBufs + dst) * 2 + 1] = cf;
    b.nfullEnd[p * kOdBufs + dst] = cu;
    if (mode != 0) {  // laserCloudCornerLastNum / SurfLastNum (:901-902); the init frame leaves 0 (Q8)
      b.istate[(size_t)p * kOdStateInts + kIsCornerLastNum] = cl;
      b.istate[(size_t)p * kOdStateInts + kIsSurfLastNum] = cf;
    }
    if (nl > b.capC || nf > b.capS || nfull > b.capS) b.istate[(size_t)p * kOdStateInts + kIsErr] |= ERR_CAP_ROWS;
  }
}

// ---------------------------------------------------------------- host side
hipError_t od_alloc(OdBuffers& b, int P, int R, int cap_pts, int max_iter) {
  DevAlloc A;
  b.P = P;
  b.capC = kLessSharpPerRing * R;
  b.capS = cap_pts;
  b.max_iter = max_iter;
  b.cap_q = (kSharpPerRing + kFlatPerRing) * R;
  b.gq = (b.cap_q + kOdThreads - 1) / kOdThreads;
  b.tC = next_pow2(b.capC);
  b.tS = next_pow2(b.capS) > 65536 ? 65536 : next_pow2(b.capS);
  A(&b.state_set[0], (size_t)P * kOdStateFloats * sizeof(float));
  A(&b.state_set[1], (size_t)P * kOdStateFloats * sizeof(float));
  A(&b.state_set[2], (size_t)P * kOdStateFloats * sizeof(float));
  b.state = b.state_set[0];
  A(&b.istate_set[0], (size_t)P * kOdStateInts * sizeof(int));
  A(&b.istate_set[1], (size_t)P * kOdStateInts * sizeof(int));
  A(&b.istate_set[2], (size_t)P * kOdStateInts * sizeof(int));
  b.istate = b.istate_set[0];
  A(&b.lastC, (size_t)kOdBufs * P * b.capC * sizeof(float4));
  A(&b.lastS, (size_t)kOdBufs * P * b.capS * sizeof(float4));
  A(&b.fullEnd, (size_t)kOdBufs * P * b.capS * sizeof(float4));
  A(&b.nlast, (size_t)P * kOdBufs * 2 * sizeof(int));
  A(&b.nfullEnd, (size_t)P * kOdBufs * sizeof(int));
  A(&b.hC_start, (size_t)kOdBufs * P * (b.tC + 1) * sizeof(int));
  A(&b.hS_start, (size_t)kOdBufs * P * (b.tS + 1) * sizeof(int));
  A(&b.hC_fill, (size_t)P * b.tC * sizeof(int));
  A(&b.hS_fill, (size_t)P * b.tS * sizeof(int));
  A(&b.hC_pts, (size_t)kOdBufs * P * b.capC * sizeof(float4));
  A(&b.hS_pts, (size_t)kOdBufs * P * b.capS * sizeof(float4));
  A(&b.hC_T, (size_t)kOdBufs * P * sizeof(int));
  A(&b.cC, (size_t)kOdBufs * P * 2 * chunks_of(b.capC) * sizeof(float4));
  A(&b.cS, (size_t)kOdBufs * P * 2 * chunks_of(b.capS) * sizeof(float4));
  A(&b.fC, (size_t)kOdBufs * P * 2 * subs_of(b.capC) * sizeof(float4));
  A(&b.fS, (size_t)kOdBufs * P * 2 * subs_of(b.capS) * sizeof(float4));
  A(&b.hS_T, (size_t)kOdBufs * P * sizeof(int));
  A(&b.ind, (size_t)P * 3 * b.cap_q * sizeof(int));
  A(&b.sel, (size_t)P * b.cap_q * sizeof(float4));
  A(&b.q_cf, (size_t)P * max_iter * b.cap_q * sizeof(float4));
  A(&b.q_ok, (size_t)P * max_iter * b.cap_q * sizeof(int8_t));
  A(&b.mom, (size_t)P * kOdMom * b.cap_q * sizeof(double));
  A(&b.qa, (size_t)P * b.cap_q * 3 * sizeof(float4));
  // per-workgroup partials: [P][gq][28], or [P][gq * max_iter][28] for the small-batch rows kernel
  A(&b.part, (size_t)P * b.gq * max_iter * 28 * sizeof(double));  // (k_od_rows_small: per stored iteration)
  A(&b.done, (size_t)P * sizeof(int));
  A(&b.ls_part, (size_t)2 * kOdLsMaxG * 28 * sizeof(double));
  A(&b.ls_flag, (size_t)kOdLsMaxG * sizeof(unsigned long long));
  A(&b.ls_epoch, sizeof(unsigned long long));
  A(&b.mono, (size_t)kOdBufs * P * 2 * sizeof(int));
  A(&b.rstart, (size_t)kOdBufs * P * 2 * kRingTab * sizeof(int));
  if (A.err != hipSuccess) {
    od_free(b);
    return A.err;
  }
  if (A.err == hipSuccess) A.err = hipMemset(b.done, 0, (size_t)P * sizeof(int));
  if (A.err == hipSuccess) A.err = hipMemset(b.ls_flag, 0, (size_t)kOdLsMaxG * sizeof(unsigned long long));
  if (A.err == hipSuccess) A.err = hipMemset(b.ls_epoch, 0, sizeof(unsigned long long));
  for (int k = 0; k < 3; ++k)
    if (A.err == hipSuccess) A.err = hipMemset(b.state_set[k], 0, (size_t)P * kOdStateFloats * sizeof(float));
  for (int k = 0; k < 3; ++k)
    if (A.err == hipSuccess) A.err = hipMemset(b.istate_set[k], 0, (size_t)P * kOdStateInts * sizeof(int));
  if (A.err == hipSuccess) A.err = hipMemset(b.nlast, 0, (size_t)P * kOdBufs * 2 * sizeof(int));
  if (A.err == hipSuccess) A.err = hipMemset(b.nfullEnd, 0, (size_t)P * kOdBufs * sizeof(int));
  if (A.err == hipSuccess) A.err = hipMemset(b.hC_T, 0, (size_t)kOdBufs * P * sizeof(int));
  if (A.err == hipSuccess) A.err = hipMemset(b.hS_T, 0, (size_t)kOdBufs * P * sizeof(int));
  if (A.err != hipSuccess) od_free(b);
  return A.err;
}

void od_free(OdBuffers& b) {
  if (b.hash_pending && b.hash_done) (void)hipEventSynchronize(b.hash_done);
  if (b.hash_fork) (void)hipEventDestroy(b.hash_fork);
  if (b.hash_done) (void)hipEventDestroy(b.hash_done);
  void* ptrs[] = {b.state_set[0], b.state_set[1], b.state_set[2], b.istate_set[0], b.istate_set[1], b.istate_set[2], b.lastC, b.lastS, b.fullEnd, b.nlast, b.nfullEnd, b.hC_start,
                  b.hS_start, b.hC_fill, b.hS_fill, b.hC_pts, b.hS_pts, b.hC_T, b.hS_T, b.cC, b.cS,
                  b.ind, b.sel, b.q_cf, b.q_ok, b.mom, b.qa, b.part, b.done, b.mono, b.rstart, b.fC, b.fS,
                  b.ls_part, b.ls_flag, b.ls_epoch};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  b = OdBuffers();
}

// voxel hashes of Last[buf] (corner and surf), 1 m cells
hipError_t od_build_hashes_deferred(OdBuffers& b, int buf, hipStream_t st, hipStream_t side) {
  hipError_t e = hipSuccess;
  if (!b.hash_fork) e = hipEventCreateWithFlags(&b.hash_fork, hipEventDisableTiming);
  if (e == hipSuccess && !b.hash_done) e = hipEventCreateWithFlags(&b.hash_done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(b.hash_fork, st);
  if (e == hipSuccess) e = hipStreamWaitEvent(side, b.hash_fork, 0);
  if (e != hipSuccess) return e;
  od_build_hashes(b, buf, side);
  e = hipEventRecord(b.hash_done, side);
  if (e == hipSuccess) b.hash_pending = true;
  return e;
}

hipError_t od_wait_hashes(OdBuffers& b, hipStream_t st) {
  if (!b.hash_pending) return hipSuccess;
  b.hash_pending = false;
  return hipStreamWaitEvent(st, b.hash_done, 0);
}

void od_build_hashes(const OdBuffers& b, int buf, hipStream_t st) {
  HashJob jc;
  jc.pts = b.lastC + (size_t)buf * b.P * b.capC;
  jc.pts_stride = b.capC;
  jc.pts_off = nullptr;
  jc.pts_off_stride = 0;
  jc.count = b.nlast + buf * 2 + 0;
  jc.count_stride_bytes = 2 * kOdBufs * sizeof(int);
  jc.start = b.hC_start + (size_t)buf * b.P * (b.tC + 1);
  jc.fill = b.hC_fill;
  jc.out = b.hC_pts + (size_t)buf * b.P * b.capC;
  jc.tsize = b.hC_T + buf * b.P;
  jc.tmax = b.tC;
  jc.inv_h = 1.0f;
  jc.shift = 1;
  jc.chunks = b.cC + (size_t)buf * b.P * 2 * chunks_of(b.capC);
  jc.fine = b.fC + (size_t)buf * b.P * 2 * subs_of(b.capC);
  jc.mono = b.mono + (size_t)buf * b.P * 2;
  jc.mono_stride = 2;
  jc.rstart = b.rstart + (size_t)buf * b.P * 2 * kRingTab;
  jc.rstart_stride = 2 * kRingTab;
  HashJob js = jc;
  js.mono = jc.mono + 1;
  js.rstart = jc.rstart + kRingTab;
  js.pts = b.lastS + (size_t)buf * b.P * b.capS;
  js.pts_stride = b.capS;
  js.count = b.nlast + buf * 2 + 1;
  js.start = b.hS_start + (size_t)buf * b.P * (b.tS + 1);
  js.fill = b.hS_fill;
  js.out = b.hS_pts + (size_t)buf * b.P * b.capS;
  js.tsize = b.hS_T + buf * b.P;
  js.tmax = b.tS;
  js.chunks = b.cS + (size_t)buf * b.P * 2 * chunks_of(b.capS);
  js.fine = b.fS + (size_t)buf * b.P * 2 * subs_of(b.capS);
  hash_build_pair(jc, js, b.P, st, true);
}

}  // namespace loam

namespace loam {
void od_solve(const OdBuffers& b, const FeatView& f, int last_buf, hipStream_t st, Prof* prof, bool device_fini) {
  const int P = b.P;
  auto mark = [&](const char* n) { if (prof) prof->mark(n); };
  hipLaunchKernelGGL(k_od_begin, dim3((P + 255) / 256), dim3(256), 0, st, b, f);
  const Tuning& tn = b.tune;
  // one problem (streaming): the whole L-M loop as one persistent launch (tuning od_persist)
  const int gls = P == 1 && tn.od_persist ? od_lm_stream_grid(b.cap_q) : 0;
  if (gls > 0) {
    hipLaunchKernelGGL(k_od_lm_stream, dim3(gls), dim3(kOdLsThreads), 0, st, b, f, last_buf);
    mark("k_od_lm_stream");
  }
  for (int it = 0; it < (gls > 0 ? 0 : b.max_iter); ++it) {
    if (it % 5 == 0) {  // Q10
      // one wave per query when the batch is small (streaming: TransformToStart in the wave), 64
      // waves per problem otherwise (the queries transformed by k_od_sel first)
      // (batches: about nine query capacity per wave — 64 waves per VLP-16 problem, 256 per HDL-64E
      // one; round 5, config 5: 64 -> 256 waves took k_od_assoc 4.09 -> 2.48 ms/step, while at
      // VLP-16 batches 32 / 128 / 256 measured equal / slower)
      const int ga = P >= 64 ? (tn.od_assoc_wg > 0 ? tn.od_assoc_wg : std::max(16, std::min(1024, b.cap_q / 9)))
                             : (b.cap_q + kAsWaves - 1) / kAsWaves;
      if (P >= tn.od_sel_min) {
        hipLaunchKernelGGL(k_od_sel, dim3(b.gq, P), dim3(kOdThreads), 0, st, b, f);
        if (prof) {
          hipLaunchKernelGGL((k_od_assoc<true, false>), dim3(ga, P), dim3(kAsThreads), 0, st, b, f, last_buf);
        } else {
          hipLaunchKernelGGL((k_od_assoc<false, false>), dim3(ga, P), dim3(kAsThreads), 0, st, b, f, last_buf);
        }
      } else {
        if (prof) hipLaunchKernelGGL((k_od_assoc<true, true>), dim3(ga, P), dim3(kAsThreads), 0, st, b, f, last_buf);
        else hipLaunchKernelGGL((k_od_assoc<false, true>), dim3(ga, P), dim3(kAsThreads), 0, st, b, f, last_buf);
      }
      mark("k_od_assoc");
    }
    if (P <= tn.od_small_max) {  // measured: the fused step loses for large batches (its serial tail)
      hipLaunchKernelGGL(k_od_rows_small, dim3(b.gq, P, it + 1), dim3(kOdThreads), 0, st, b, f, last_buf, it);
      mark("k_od_rows");
    } else {
      const bool mom = P >= tn.od_moments_min;     // the stored rows as per-query moments (not bit-exact)
      if (P <= tn.od_fused_max) {
        if (mom) hipLaunchKernelGGL((k_od_rows_mom<true>), dim3(b.gq, P), dim3(kOdThreads), 0, st, b, f, last_buf, it);
        else hipLaunchKernelGGL((k_od_rows<true, 2>), dim3(b.gq, P), dim3(kOdThreads), 0, st, b, f, last_buf, it);
        mark("k_od_rows");
      } else {
        if (mom) hipLaunchKernelGGL((k_od_rows_mom<false>), dim3(b.gq, P), dim3(kOdThreads), 0, st, b, f, last_buf, it);
        else hipLaunchKernelGGL((k_od_rows<false, 2>), dim3(b.gq, P), dim3(kOdThreads), 0, st, b, f, last_buf, it);
        mark("k_od_rows");
        hipLaunchKernelGGL(k_od_step, dim3(P), dim3(64), 0, st, b, it, b.gq);
        mark("k_od_step");
      }
    }
  }
  if (device_fini) hipLaunchKernelGGL(k_od_fini, dim3((P + 63) / 64), dim3(64), 0, st, b, f);
}

void od_fini(const OdBuffers& b, const FeatView& f, hipStream_t st) {
  hipLaunchKernelGGL(k_od_fini, dim3((b.P + 63) / 64), dim3(64), 0, st, b, f);
}
}  // namespace loam


#ifdef LOAM_PHASES
// the phase sums of the last-workgroup kernel of this file (PhaseAcc, dev_common.hpp); diagnostic
// build only (tools/phase_stream.py)
extern "C" int loam_debug_phases_od(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(loam::g_ph_od), sizeof(PhaseAcc)) == hipSuccess ? 0 : -1;
}
#endif
