// Scan registration on gfx950: laserCloudHandler (/root/reference/src/scanRegistration.cpp:211-636)
// as four kernels over a batch of sweeps.
//
//  k_sr_ring_sort   one workgroup per sweep: NaN filter, axis swap, ring ID, orientation with the
//                   sequential halfPassed flag (a block min-reduction finds the flip point), relTime,
//                   intensity, stable ring bucketing (per-tile ring counts + wave ballot ranks).
//                   src/scanRegistration.cpp:225-357
//  k_sr_features    256-point tiles with a 6-point halo in LDS: 11-tap curvature, ring bounds
//                   (last-write-wins transitions = atomicMax), occlusion / parallel-beam marks as a
//                   gather over the 12 neighbouring events.  :358-452
//  k_sr_select      one workgroup per (sweep, ring): the six segment sorts as one LDS bitonic sort
//                   of the ring by (segment, curvature, position) = the reference's stable
//                   insertion sorts, the greedy sharp / flat picks and lessFlat candidates by one
//                   wave with ballots on LDS state (the neighbour-walk distance tests are
//                   precomputed gap bits), PCL VoxelGrid 0.2 of the ring (LDS sort by (voxel,
//                   position), ordered per-voxel sums).  :460-581
//                   Rings are independent whenever their spans are >5 points apart (always for
//                   sweeps with no empty ring); otherwise one workgroup walks the rings in order.
//  k_sr_compact     per sweep: ring-major concatenation of the picks and the downsampled lessFlat.
//
// HBM traffic per sweep (algorithmic): 16 B/pt raw read, 16 B/pt ring-sorted
// write + read, 16 B per feature point written.
#include <type_traits>

#include "dev_common.hpp"
#include "engine.hpp"

using namespace loamdev;

namespace loam {

namespace {


LOAM_D int ring_id(const SrParams& p, float angle) {
  if (p.ring_model == LOAM_RING_LINEAR) {
    const float step = (p.ring_hi - p.ring_lo) / (float)(p.R - 1);
    const float angleID = (angle - p.ring_lo) / step;
    return (int)(angleID + 0.5f);
  }
  int rounded = (int)(D(angle) + (D(angle) < 0.0 ? -0.5 : +0.5));
  return rounded > 0 ? rounded : rounded + (p.R - 1);
}

// The reference computes the vertical angle in double (:241-247).  The float evaluation is within
// 1e-4 degrees of it, so whenever a +-1e-3 degree bracket around it maps to one ring the double
// evaluation cannot land elsewhere; only points that close to a ring boundary pay for it.
LOAM_D int ring_of(const SrParams& p, float px, float py, float pz) {
  const float af = atanf(py / sqrtf(px * px + pz * pz)) * 57.2957795f;
  const int lo = ring_id(p, af - 1e-3f), hi = ring_id(p, af + 1e-3f);
  if (lo == hi) return lo;
  return ring_id(p, (float)(atan(D(py) / sqrt(D(px * px + pz * pz))) * 180 / M_PI));
}

LOAM_D float ori_first(float ori, float startOri) {  // :263-268
  if (D(ori) < D(startOri) - M_PI / 2) ori = (float)(D(ori) + 2 * M_PI);
  else if (D(ori) > D(startOri) + M_PI * 3 / 2) ori = (float)(D(ori) - 2 * M_PI);
  return ori;
}
LOAM_D float ori_second(float ori, float endOri) {  // :274-280
  ori = (float)(D(ori) + 2 * M_PI);
  if (D(ori) < D(endOri) - M_PI * 3 / 2) ori = (float)(D(ori) + 2 * M_PI);
  else if (D(ori) > D(endOri) + M_PI / 2) ori = (float)(D(ori) - 2 * M_PI);
  return ori;
}
LOAM_D bool finite3(const float4& q) {
  return isfinite(q.x) && isfinite(q.y) && isfinite(q.z);
}

// ---------------------------------------------------------------- ring sort
template <bool IMU>
__global__ __launch_bounds__(kSrThreads) void k_sr_ring_sort(SrBuffers b, SrParams p) {
  const int s = blockIdx.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int n = b.raw_n[s];
  const float4* raw = b.raw + (size_t)s * b.cap;
  float* tori = b.tmp_ori + (size_t)s * b.cap;
  uint8_t* tsid = b.tmp_sid + (size_t)s * b.cap;
  const int R = p.R, ntiles = (n + kSrThreads - 1) / kSrThreads;
  int* tc = b.tilecnt + (size_t)s * b.ntiles() * R;
  __shared__ int sh_first, sh_last, sh_F, sh_total;
  __shared__ float sh_start, sh_end;
  __shared__ int sh_cnt[64];
  __shared__ int sh_wcnt[kSrThreads / 64][64];
  __shared__ int sh_base[64];
  if (tid == 0) { sh_first = 0x7fffffff; sh_last = -1; sh_F = 0x7fffffff; }
  __syncthreads();
  int f = 0x7fffffff, l = -1;
  for (int i = tid; i < n; i += kSrThreads) {
    if (finite3(raw[i])) { f = min(f, i); l = max(l, i); }
  }
  f = wave_min_i(f);
  l = wave_max_i(l);
  if (lane == 0) { atomicMin(&sh_first, f); atomicMax(&sh_last, l); }
  __syncthreads();
  if (sh_last < 0) {
    if (tid == 0) { b.n_full[s] = 0; b.err[s] |= ERR_EMPTY; }
    return;
  }
  if (tid == 0) {  // :230-238
    float4 a = raw[sh_first], z = raw[sh_last];
    float startOri = -atan2f_fdlibm(a.y, a.x);
    float endOri = (float)(D(-atan2f_fdlibm(z.y, z.x)) + 2 * M_PI);
    if (D(endOri - startOri) > 3 * M_PI) endOri = (float)(D(endOri) - 2 * M_PI);
    else if (D(endOri - startOri) < M_PI) endOri = (float)(D(endOri) + 2 * M_PI);
    sh_start = startOri;
    sh_end = endOri;
  }
  __syncthreads();
  const float startOri = sh_start, endOri = sh_end;
  // phase A: ring id + first-branch orientation; the halfPassed flip point F
  int Floc = 0x7fffffff;
  for (int t = 0; t < ntiles; ++t) {
    if (tid < R) sh_cnt[tid] = 0;
    __syncthreads();
    const int i = t * kSrThreads + tid;
    if (i < n) {
      const float4 q = raw[i];
      uint8_t sid = 255;
      float ori = 0.0f;
      if (finite3(q)) {
        const float px = q.y, py = q.z, pz = q.x;
        int scanID = ring_of(p, px, py, pz);
        if (scanID >= 0 && scanID <= R - 1) {
          sid = (uint8_t)scanID;
          ori = -atan2f_fdlibm(px, pz);
          float o1 = ori_first(ori, startOri);
          if (D(o1 - startOri) > M_PI) Floc = min(Floc, i);
          atomicAdd(&sh_cnt[scanID], 1);
        }
      }
      tori[i] = ori;
      tsid[i] = sid;
    }
    __syncthreads();
    if (tid < R) tc[t * R + tid] = sh_cnt[tid];
    __syncthreads();
  }
  Floc = wave_min_i(Floc);
  if (lane == 0) atomicMin(&sh_F, Floc);
  __threadfence_block();
  __syncthreads();
  // phase B: per-ring exclusive scan over tiles, ring bases
  if (tid < R) {
    int run = 0;
    for (int t = 0; t < ntiles; ++t) {
      int c = tc[t * R + tid];
      tc[t * R + tid] = run;
      run += c;
    }
    sh_cnt[tid] = run;
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int r = 0; r < R; ++r) { sh_base[r] = run; run += sh_cnt[r]; }
    sh_total = run;
  }
  __syncthreads();
  const int F = sh_F;
  // IMU (:286-349, sweep 0 of a streaming context only): the Start state from the first finite
  // point when it passed the ring filter (the reference's i == 0), else the previous sweep's
  loamimu::SrQueue* imu = IMU && s == 0 ? p.imu : nullptr;
  __shared__ loamimu::Start sh_S;
  __shared__ int sh_carry, sh_imuscr[kSrThreads / 64 + 1], sh_lasti;
  __shared__ loamimu::Cur sh_lastc;
  __shared__ float sh_lastfs[6];
  const int i0 = sh_first;
  const int front0 = imu ? imu->front : 0;
  if (imu && tid == 0) {
    loamimu::Cur c;
    if (tsid[i0] != 255) {
      const float ori = ori_first(tori[i0], startOri);  // i0 <= F
      const float relTime = (ori - startOri) / (endOri - startOri);
      const float pointTime = (float)(D(relTime) * 0.1);  // scanPeriod (double, :55)
      const int g = loamimu::first_later(*imu, front0, p.time_scan + pointTime);
      c = loamimu::interpolate(*imu, (front0 + g) % loamimu::kQue, p.time_scan, pointTime);
      imu->rollStart = c.roll; imu->pitchStart = c.pitch; imu->yawStart = c.yaw;
      imu->veloXStart = c.vx; imu->veloYStart = c.vy; imu->veloZStart = c.vz;
      imu->shiftXStart = c.sx; imu->shiftYStart = c.sy; imu->shiftZStart = c.sz;
    } else {
      c = loamimu::Cur{imu->rollStart, imu->pitchStart, imu->yawStart, imu->veloXStart, imu->veloYStart,
                       imu->veloZStart, imu->shiftXStart, imu->shiftYStart, imu->shiftZStart};
    }
    sh_S = loamimu::make_start(c);
    sh_carry = 0;
    sh_lasti = -1;
  }
  __syncthreads();
  // phase C: stable scatter into ring order
  for (int t = 0; t < ntiles; ++t) {
    const int i = t * kSrThreads + tid;
    int sid = 255;
    if (i < n) sid = tsid[i];
    const bool valid = (i < n) && sid != 255;
    // IMU queue entry of every point: the reference's forward-only pointer walk (:288-293) is the
    // running maximum, over the points in input order, of "first entry later than the point"
    float pointTime = 0.0f;
    int front_i = 0;
    if (imu) {
      int g = -1;
      if (valid) {
        const float ori = (i <= F) ? ori_first(tori[i], startOri) : ori_second(tori[i], endOri);
        const float relTime = (ori - startOri) / (endOri - startOri);
        pointTime = (float)(D(relTime) * 0.1);
        g = loamimu::first_later(*imu, front0, p.time_scan + pointTime);
      }
      int tmax;
      const int incl = block_incl_max<kSrThreads>(g, sh_imuscr, tmax);
      front_i = max(sh_carry, incl);
      __syncthreads();
      if (tid == 0) sh_carry = max(sh_carry, tmax);
    }
    loamimu::Cur cur;
    float fs[6];
    if (lane < R) sh_wcnt[w][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    int rank = 0;
    uint64_t mval = __ballot(valid);
    while (mval) {
      const int leader = __ffsll((unsigned long long)mval) - 1;
      const int rl = __builtin_amdgcn_readlane(sid, leader);
      const uint64_t mm = __ballot(valid && sid == rl);
      if (valid && sid == rl) rank = __popcll(mm & lanemask_lt());
      if (lane == leader) sh_wcnt[w][rl] = __popcll(mm);
      mval &= ~mm;
    }
    __syncthreads();
    if (valid) {
      int pos = sh_base[sid] + tc[t * R + sid] + rank;
      for (int v = 0; v < w; ++v) pos += sh_wcnt[v][sid];
      const float4 q = raw[i];
      float ori = tori[i];
      ori = (i <= F) ? ori_first(ori, startOri) : ori_second(ori, endOri);
      float relTime = (ori - startOri) / (endOri - startOri);
      float4 o;
      o.x = q.y;
      o.y = q.z;
      o.z = q.x;
      o.w = (float)(sid + 0.1 * D(relTime));
      if (imu) {
        cur = loamimu::interpolate(*imu, (front0 + front_i) % loamimu::kQue, p.time_scan, pointTime);
        if (i != i0) {  // ShiftToStartIMU, VeloToStartIMU, TransformToStartIMU (:343-347)
          loamimu::to_start(sh_S, cur, pointTime, fs);
          o = loamimu::transform_to_start(sh_S, cur, fs, o);
        }
      }
      b.full[(size_t)s * b.cap + pos] = o;
    }
    if (imu) {  // the last processed point leaves its Cur / FromStart values in the globals
      int lm;
      (void)block_incl_max<kSrThreads>(valid ? i : -1, sh_imuscr, lm);
      if (valid && i == lm) {
        sh_lasti = i;
        sh_lastc = cur;
        for (int k = 0; k < 6; ++k) sh_lastfs[k] = fs[k];
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    b.n_full[s] = sh_total;
    if (imu) {
      imu->front = (front0 + sh_carry) % loamimu::kQue;
      if (sh_lasti >= 0) {
        const loamimu::Cur& c = sh_lastc;
        imu->rollCur = c.roll; imu->pitchCur = c.pitch; imu->yawCur = c.yaw;
        imu->veloXCur = c.vx; imu->veloYCur = c.vy; imu->veloZCur = c.vz;
        imu->shiftXCur = c.sx; imu->shiftYCur = c.sy; imu->shiftZCur = c.sz;
        if (sh_lasti != i0) {
          imu->shiftFSX = sh_lastfs[0]; imu->shiftFSY = sh_lastfs[1]; imu->shiftFSZ = sh_lastfs[2];
          imu->veloFSX = sh_lastfs[3]; imu->veloFSY = sh_lastfs[4]; imu->veloFSZ = sh_lastfs[5];
        }
      }
    }
  }
}

// ---------------------------------------------------------------- ring sort, tile-parallel
// The same stable ring bucketing as k_sr_ring_sort for sweeps without IMU data, one workgroup per
// kSrThreads-point tile instead of one per sweep (a single sweep then spreads over ~60 CUs instead
// of walking its tiles on one): k_sr_ring_count finds the sweep's first / last finite point itself
// (waves 0 / 1 scan from either end), computes ring ID and first-branch orientation of its tile,
// the tile's ring counts and its first halfPassed flip; k_sr_ring_scatter takes the flip point F
// as the minimum over the tiles, the ring bases and its tile's per-ring offsets from the counts,
// and scatters with the same wave-ballot ranks.  src/scanRegistration.cpp:225-357
// A tile is kRingE sub-tiles of kSrThreads points (each thread's kRingE loads in flight at once),
// which also cuts the per-tile fixed work (sweep ends, start orientation, tile prefix) kRingE-fold.
#ifndef LOAM_RING_E
#define LOAM_RING_E 4
#endif
constexpr int kRingE = LOAM_RING_E;
constexpr int kRingTile = kSrThreads * kRingE;

__global__ __launch_bounds__(kSrThreads) void k_sr_ring_count(SrBuffers b, SrParams p) {
  const int s = blockIdx.y, t = blockIdx.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int n = b.raw_n[s], R = p.R;
  if (t == 0) {  // the sweep's error bits and ring bounds start here (tile 0 alone writes err in this launch)
    if (tid < 2 * R) b.ring_se[s * 2 * R + tid] = 0;
    if (tid == 0) b.err[s] = 0;
  }
  if (t * kRingTile >= n) return;
  const float4* raw = b.raw + (size_t)s * b.cap;
  __shared__ int sh_first, sh_last, sh_F;
  __shared__ float sh_start, sh_end_raw;
  __shared__ int sh_cnt[64];
  // the tile's points first: their loads are in flight during the sweep-end scans and the start
  // orientation below
  float4 q[kRingE];
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const int i = t * kRingTile + e * kSrThreads + tid;
    q[e] = i < n ? raw[i] : make_float4(0, 0, 0, 0);
  }
  if (w == 0) {
    int f = -1;
    for (int base = 0; base < n; base += 64) {
      const int i = base + lane;
      const uint64_t m = __ballot(i < n && finite3(raw[i]));
      if (m) { f = base + __ffsll((unsigned long long)m) - 1; break; }
    }
    if (lane == 0) sh_first = f;
  } else if (w == 1) {
    int l = -1;
    for (int base = n - 1; base >= 0; base -= 64) {
      const int i = base - lane;
      const uint64_t m = __ballot(i >= 0 && finite3(raw[i]));
      if (m) { l = base - (__ffsll((unsigned long long)m) - 1); break; }
    }
    if (lane == 0) sh_last = l;
  }
  if (tid < R) sh_cnt[tid] = 0;
  if (tid == 0) sh_F = 0x7fffffff;
  __syncthreads();
  // :230-238, the two orientations on two waves; only tile 0 needs endOri
  if (tid == 0) sh_start = sh_last >= 0 ? -atan2f_fdlibm(raw[sh_first].y, raw[sh_first].x) : 0.0f;
  if (tid == 64 && t == 0 && sh_last >= 0) sh_end_raw = -atan2f_fdlibm(raw[sh_last].y, raw[sh_last].x);
  __syncthreads();
  const float startOri = sh_start;
  if (tid == 0 && t == 0) {
    float endOri = 0.0f;
    if (sh_last >= 0) {
      endOri = (float)(D(sh_end_raw) + 2 * M_PI);
      if (D(endOri - startOri) > 3 * M_PI) endOri = (float)(D(endOri) - 2 * M_PI);
      else if (D(endOri - startOri) < M_PI) endOri = (float)(D(endOri) + 2 * M_PI);
    } else {
      b.err[s] |= ERR_EMPTY;
    }
    b.sweep_ori[2 * s] = startOri;
    b.sweep_ori[2 * s + 1] = endOri;
  }
  int Floc = 0x7fffffff;
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const int i = t * kRingTile + e * kSrThreads + tid;
    if (i < n) {
      uint8_t sid = 255;
      float ori = 0.0f;
      if (finite3(q[e])) {
        const float px = q[e].y, py = q[e].z, pz = q[e].x;
        const int scanID = ring_of(p, px, py, pz);
        if (scanID >= 0 && scanID <= R - 1) {
          sid = (uint8_t)scanID;
          ori = -atan2f_fdlibm(px, pz);
          const float o1 = ori_first(ori, startOri);
          if (D(o1 - startOri) > M_PI) Floc = min(Floc, i);
          atomicAdd(&sh_cnt[scanID], 1);
        }
      }
      b.tmp_ori[(size_t)s * b.cap + i] = ori;
      b.tmp_sid[(size_t)s * b.cap + i] = sid;
    }
  }
  Floc = wave_min_i(Floc);
  if (lane == 0 && Floc != 0x7fffffff) atomicMin(&sh_F, Floc);
  __syncthreads();
  if (tid < R) b.tilecnt[((size_t)s * b.ntiles() + t) * R + tid] = sh_cnt[tid];
  if (tid == 0) b.tileF[(size_t)s * b.ntiles() + t] = sh_F;
}

__global__ __launch_bounds__(kSrThreads) void k_sr_ring_scatter(SrBuffers b, SrParams p) {
  constexpr int kW = kSrThreads / 64, kSlots = kRingE * kW;  // (sub-tile, wave) slots in point order
  static_assert(kSlots <= 64 && (kSlots & (kSlots - 1)) == 0, "slot scan width");
  const int s = blockIdx.y, t = blockIdx.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int n = b.raw_n[s], R = p.R, nt = (n + kRingTile - 1) / kRingTile;
  if (t >= (nt > 0 ? nt : 1)) return;
  __shared__ int sh_tot[64], sh_pre[64], sh_base[64], sh_F;
  __shared__ int sh_wcnt[64][kSlots];  // per ring: points of each slot, then their exclusive prefix
  // the tile's ring IDs, points and orientations first: their loads are in flight during the tile
  // prefix below (a point whose ring ID turns out invalid is loaded for nothing: rare)
  int sid[kRingE], rank[kRingE];
  float4 q[kRingE];
  float ori[kRingE];
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const int i = t * kRingTile + e * kSrThreads + tid;
    sid[e] = 255;
    q[e] = make_float4(0, 0, 0, 0);
    ori[e] = 0.0f;
    if (i < n) {
      sid[e] = (int)b.tmp_sid[(size_t)s * b.cap + i];
      q[e] = b.raw[(size_t)s * b.cap + i];
      ori[e] = b.tmp_ori[(size_t)s * b.cap + i];
    }
  }
  if (tid < R) { sh_tot[tid] = 0; sh_pre[tid] = 0; }
  if (tid == 0) sh_F = 0x7fffffff;
  for (int k = tid; k < 64 * kSlots; k += kSrThreads) (&sh_wcnt[0][0])[k] = 0;
  __syncthreads();
  const int* tc = b.tilecnt + (size_t)s * b.ntiles() * R;
  for (int k = tid; k < nt * R; k += kSrThreads) {
    const int v = tc[k];
    if (v) {
      atomicAdd(&sh_tot[k % R], v);
      if (k / R < t) atomicAdd(&sh_pre[k % R], v);
    }
  }
  int F = 0x7fffffff;
  for (int k = tid; k < nt; k += kSrThreads) F = min(F, b.tileF[(size_t)s * b.ntiles() + k]);
  F = wave_min_i(F);
  if (lane == 0 && F != 0x7fffffff) atomicMin(&sh_F, F);
  // stable ranks within each (sub-tile, wave) slot by wave ballots
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const bool valid = sid[e] != 255;
    rank[e] = 0;
    uint64_t mval = __ballot(valid);
    while (mval) {
      const int leader = __ffsll((unsigned long long)mval) - 1;
      const int rl = __builtin_amdgcn_readlane(sid[e], leader);
      const uint64_t mm = __ballot(valid && sid[e] == rl);
      if (valid && sid[e] == rl) rank[e] = __popcll(mm & lanemask_lt());
      if (lane == leader) sh_wcnt[rl][e * kW + w] = __popcll(mm);
      mval &= ~mm;
    }
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int r = 0; r < R; ++r) { sh_base[r] = run; run += sh_tot[r]; }
    if (t == 0) {
      b.n_full[s] = run;
      if (n <= 0) b.err[s] |= ERR_EMPTY;
    }
  }
  // per ring, exclusive prefix over the slots: kSlots lanes per ring, groups aligned to kSlots
  for (int k = tid; k < R * kSlots; k += kSrThreads) {
    const int r = k / kSlots, j = k % kSlots;
    const int v = sh_wcnt[r][j];
    int incl = v;
#pragma unroll
    for (int o = 1; o < kSlots; o <<= 1) {
      const int u = __shfl_up(incl, o, kSlots);
      if (j >= o) incl += u;
    }
    sh_wcnt[r][j] = incl - v;
  }
  __syncthreads();
  if (nt == 0) return;
  F = sh_F;
  const float startOri = b.sweep_ori[2 * s], endOri = b.sweep_ori[2 * s + 1];
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const int i = t * kRingTile + e * kSrThreads + tid;
    if (sid[e] != 255) {
      const int pos = sh_base[sid[e]] + sh_pre[sid[e]] + sh_wcnt[sid[e]][e * kW + w] + rank[e];
      const float o = (i <= F) ? ori_first(ori[e], startOri) : ori_second(ori[e], endOri);
      const float relTime = (o - startOri) / (endOri - startOri);
      b.full[(size_t)s * b.cap + pos] = make_float4(q[e].y, q[e].z, q[e].x, (float)(sid[e] + 0.1 * D(relTime)));
    }
  }
}

// The ring count and scatter in one launch, each raw point read once and held in registers from
// its ring ID to its store (no tmp_ori / tmp_sid round trip, no second raw read).  A tile counts
// its rings and its first flip, publishes them (tilecnt / tileF, [S][rtiles] rows here), ranks its
// points by wave ballots while the sweep's other tiles count, waits for all of them, and
// scatters.  Tiles take tickets in launch order (ring_sync[0]) and a sweep's tiles hold
// consecutive tickets, so every tile a waiting tile needs has started: only the last sweep under
// way can still be short of tiles, and the other resident tiles finish and free their slots.
#ifndef LOAM_SR_RING_FUSED
#define LOAM_SR_RING_FUSED 1
#endif
constexpr bool kSrRingFused = LOAM_SR_RING_FUSED;
// ... for launches of at least this many sweeps (its three presets are launches of their own: a
// one-sweep chain keeps the two-kernel form)
constexpr int kSrRingFusedMin = 64;
__global__ __launch_bounds__(kSrThreads) void k_sr_ring_fused(SrBuffers b, SrParams p, int rtiles) {
  constexpr int kW = kSrThreads / 64, kSlots = kRingE * kW;
  static_assert(kSlots <= 64 && (kSlots & (kSlots - 1)) == 0, "slot scan width");
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  __shared__ int sh_ticket, sh_last, sh_F;
  __shared__ float sh_start, sh_end_raw;
  __shared__ int sh_cnt[64], sh_tot[64], sh_pre[64], sh_base[64];
  __shared__ int sh_wcnt[64][kSlots];
  if (tid == 0) sh_ticket = atomicAdd(&b.ring_sync[0], 1);
  __syncthreads();
  const int s = sh_ticket / rtiles, t = sh_ticket % rtiles;
  const int n = b.raw_n[s], R = p.R, nt = (n + kRingTile - 1) / kRingTile;
  if (t == 0) {  // the sweep's error bits and ring bounds start here (tile 0 alone writes err in this launch)
    if (tid < 2 * R) b.ring_se[s * 2 * R + tid] = 0;
    if (tid == 0) b.err[s] = 0;
  }
  if (n <= 0) {
    if (t == 0 && tid == 0) {
      b.n_full[s] = 0;
      b.err[s] |= ERR_EMPTY;
    }
    return;
  }
  if (t >= nt) return;
  const float4* raw = b.raw + (size_t)s * b.cap;
  float4 q[kRingE];
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const int i = t * kRingTile + e * kSrThreads + tid;
    q[e] = i < n ? raw[i] : make_float4(0, 0, 0, 0);
  }
  // :230-238's first and last finite points, scanned from either end by waves 0 / 1; the lane
  // that holds the point hands its coordinates over (no second load), -atan2 on lane 0
  if (w < 2) {
    int f = -1;
    float4 v = make_float4(0, 0, 0, 0);
    for (int k = 0; k < n; k += 64) {
      const int i = w == 0 ? k + lane : n - 1 - k - lane;
      const bool in = w == 0 ? i < n : i >= 0;
      v = in ? raw[i] : make_float4(0, 0, 0, 0);
      const uint64_t m = __ballot(in && finite3(v));
      if (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        f = w == 0 ? k + src : n - 1 - k - src;
        v.x = __shfl(v.x, src, 64);
        v.y = __shfl(v.y, src, 64);
        break;
      }
    }
    if (lane == 0) {
      if (w == 0) {
        sh_start = f >= 0 ? -atan2f_fdlibm(v.y, v.x) : 0.0f;
      } else {
        sh_last = f;
        if (f >= 0) sh_end_raw = -atan2f_fdlibm(v.y, v.x);
      }
    }
  }
  if (tid < R) sh_cnt[tid] = 0;
  if (tid == 0) sh_F = 0x7fffffff;
  for (int k = tid; k < 64 * kSlots; k += kSrThreads) (&sh_wcnt[0][0])[k] = 0;
  __syncthreads();
  const float startOri = sh_start;
  float endOri = 0.0f;
  if (sh_last >= 0) {
    endOri = (float)(D(sh_end_raw) + 2 * M_PI);
    if (D(endOri - startOri) > 3 * M_PI) endOri = (float)(D(endOri) - 2 * M_PI);
    else if (D(endOri - startOri) < M_PI) endOri = (float)(D(endOri) + 2 * M_PI);
  }
  if (tid == 0 && t == 0) {
    if (sh_last < 0) b.err[s] |= ERR_EMPTY;
    b.sweep_ori[2 * s] = startOri;
    b.sweep_ori[2 * s + 1] = endOri;
  }
  int sid[kRingE], rank[kRingE];
  float ori[kRingE];
  int Floc = 0x7fffffff;
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const int i = t * kRingTile + e * kSrThreads + tid;
    sid[e] = 255;
    ori[e] = 0.0f;
    if (i < n && finite3(q[e])) {
      const float px = q[e].y, py = q[e].z, pz = q[e].x;
      const int scanID = ring_of(p, px, py, pz);
      if (scanID >= 0 && scanID <= R - 1) {
        sid[e] = scanID;
        ori[e] = -atan2f_fdlibm(px, pz);
        if (D(ori_first(ori[e], startOri) - startOri) > M_PI) Floc = min(Floc, i);
        atomicAdd(&sh_cnt[scanID], 1);
      }
    }
  }
  Floc = wave_min_i(Floc);
  if (lane == 0 && Floc != 0x7fffffff) atomicMin(&sh_F, Floc);
  __syncthreads();
  // published with coherent single-word stores: a reader waits on each word itself (the launch
  // presets them to -1), so no fence orders them (an agent-scope fence writes back / invalidates
  // the XCD's whole L2)
  if (tid < R) __hip_atomic_store(&b.tilecnt[((size_t)s * rtiles + t) * R + tid], sh_cnt[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid == 0) __hip_atomic_store(&b.tileF[(size_t)s * rtiles + t], sh_F, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // stable ranks within each (sub-tile, wave) slot by wave ballots, while the other tiles count
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const bool valid = sid[e] != 255;
    rank[e] = 0;
    uint64_t mval = __ballot(valid);
    while (mval) {
      const int leader = __ffsll((unsigned long long)mval) - 1;
      const int rl = __builtin_amdgcn_readlane(sid[e], leader);
      const uint64_t mm = __ballot(valid && sid[e] == rl);
      if (valid && sid[e] == rl) rank[e] = __popcll(mm & lanemask_lt());
      if (lane == leader) sh_wcnt[rl][e * kW + w] = __popcll(mm);
      mval &= ~mm;
    }
  }
  if (tid < R) { sh_tot[tid] = 0; sh_pre[tid] = 0; }
  __syncthreads();
  // per ring, exclusive prefix over the slots: kSlots lanes per ring, groups aligned to kSlots
  for (int k = tid; k < R * kSlots; k += kSrThreads) {
    const int r = k / kSlots, j = k % kSlots;
    const int v = sh_wcnt[r][j];
    int incl = v;
#pragma unroll
    for (int o = 1; o < kSlots; o <<= 1) {
      const int u = __shfl_up(incl, o, kSlots);
      if (j >= o) incl += u;
    }
    sh_wcnt[r][j] = incl - v;
  }
  const int* tc = b.tilecnt + (size_t)s * rtiles * R;
  for (int k = tid; k < nt * R; k += kSrThreads) {
    int v;
    while ((v = __hip_atomic_load(&tc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < 0) __builtin_amdgcn_s_sleep(1);
    if (v) {
      atomicAdd(&sh_tot[k % R], v);
      if (k / R < t) atomicAdd(&sh_pre[k % R], v);
    }
  }
  int F = 0x7fffffff;
  for (int k = tid; k < nt; k += kSrThreads) {
    int v;
    while ((v = __hip_atomic_load(&b.tileF[(size_t)s * rtiles + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < 0)
      __builtin_amdgcn_s_sleep(1);
    F = min(F, v);
  }
  F = wave_min_i(F);
  if (tid == 0) sh_F = 0x7fffffff;
  __syncthreads();
  if (lane == 0 && F != 0x7fffffff) atomicMin(&sh_F, F);
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int r = 0; r < R; ++r) { sh_base[r] = run; run += sh_tot[r]; }
    if (t == 0) b.n_full[s] = run;
  }
  __syncthreads();
  F = sh_F;
#pragma unroll
  for (int e = 0; e < kRingE; ++e) {
    const int i = t * kRingTile + e * kSrThreads + tid;
    if (sid[e] != 255) {
      const int pos = sh_base[sid[e]] + sh_pre[sid[e]] + sh_wcnt[sid[e]][e * kW + w] + rank[e];
      const float o = (i <= F) ? ori_first(ori[e], startOri) : ori_second(ori[e], endOri);
      const float relTime = (o - startOri) / (endOri - startOri);
      b.full[(size_t)s * b.cap + pos] = make_float4(q[e].y, q[e].z, q[e].x, (float)(sid[e] + 0.1 * D(relTime)));
    }
  }
}

// ---------------------------------------------------------------- curvature + marks
constexpr int kFeatTile = 256;  // threads
constexpr int kFeatE = 4;  // points per thread
constexpr int kFeatSpan = kFeatTile * kFeatE;

__global__ __launch_bounds__(kFeatTile) void k_sr_features(SrBuffers b, SrParams p) {
  const int s = blockIdx.y, tid = threadIdx.x;
  if ((blockIdx.x | blockIdx.y) == 0 && tid < 2) b.sel_list[tid] = 0;  // (the selection's routing lists)
  const int n = b.n_full[s];
  const int i0 = blockIdx.x * kFeatSpan;
  if (i0 >= n) return;
  const float4* pts = b.full + (size_t)s * b.cap;
  __shared__ float4 sp[kFeatSpan + 12];
  __shared__ int8_t evt[kFeatSpan + 12];
  for (int t = tid; t < kFeatSpan + 12; t += kFeatTile) {
    int g = i0 - 6 + t;
    if (g >= 0 && g < n) sp[t] = pts[g];
  }
  __syncthreads();
  for (int t = tid; t < kFeatSpan + 11; t += kFeatTile) {  // occlusion events (:395-438)
    const int k = i0 - 6 + t;
    int8_t e = 0;
    if (k >= 5 && k <= n - 7) {
      const float4 a = sp[t], c = sp[t + 1];
      float dX = c.x - a.x, dY = c.y - a.y, dZ = c.z - a.z;
      float diff = dX * dX + dY * dY + dZ * dZ;
      if (D(diff) > 0.1) {
        float depth1 = (float)sqrt(D(a.x * a.x + a.y * a.y + a.z * a.z));
        float depth2 = (float)sqrt(D(c.x * c.x + c.y * c.y + c.z * c.z));
        if (depth1 > depth2) {
          dX = c.x - a.x * depth2 / depth1;
          dY = c.y - a.y * depth2 / depth1;
          dZ = c.z - a.z * depth2 / depth1;
          if (sqrt(D(dX * dX + dY * dY + dZ * dZ)) / D(depth2) < 0.1) e = 1;
        } else {
          dX = c.x * depth1 / depth2 - a.x;
          dY = c.y * depth1 / depth2 - a.y;
          dZ = c.z * depth1 / depth2 - a.z;
          if (sqrt(D(dX * dX + dY * dY + dZ * dZ)) / D(depth1) < 0.1) e = 2;
        }
      }
    }
    evt[t] = e;
  }
  __syncthreads();
#pragma unroll
  for (int fe = 0; fe < kFeatE; ++fe) {
    const int i = i0 + fe * kFeatTile + tid;
    if (i >= n) return;
    const int li = fe * kFeatTile + tid + 6;
    const size_t gi = (size_t)s * b.cap + i;
    float cv = 0.0f;
    if (i >= 5 && i < n - 5) {  // :359-378
      const float4* q = sp + li;
      float dX = q[-5].x + q[-4].x + q[-3].x + q[-2].x + q[-1].x - 10 * q[0].x + q[1].x + q[2].x +
                 q[3].x + q[4].x + q[5].x;
      float dY = q[-5].y + q[-4].y + q[-3].y + q[-2].y + q[-1].y - 10 * q[0].y + q[1].y + q[2].y +
                 q[3].y + q[4].y + q[5].y;
      float dZ = q[-5].z + q[-4].z + q[-3].z + q[-2].z + q[-1].z - 10 * q[0].z + q[1].z + q[2].z +
                 q[3].z + q[4].z + q[5].z;
      cv = dX * dX + dY * dY + dZ * dZ;
      // ring bounds (:383-390): the last transition into ring v wins
      const int v = (int)q[0].w;
      const int pv = (i == 5) ? -1 : (int)q[-1].w;
      if (v != pv && v > 0 && v < p.R) {
        atomicMax(&b.ring_se[s * 2 * p.R + v], i + 5);
        atomicMax(&b.ring_se[s * 2 * p.R + p.R + v - 1], i - 5);
      }
    }
    int pk = 0;
    for (int k = 0; k <= 5; ++k) pk |= (evt[li + k] == 1);
    for (int k = 1; k <= 6; ++k) pk |= (evt[li - k] == 2);
    if (i >= 5 && i <= n - 7) {  // :440-451
      const float4 a = sp[li - 1], c = sp[li], e = sp[li + 1];
      float dX = e.x - c.x, dY = e.y - c.y, dZ = e.z - c.z;
      float diff = dX * dX + dY * dY + dZ * dZ;
      float dX2 = c.x - a.x, dY2 = c.y - a.y, dZ2 = c.z - a.z;
      float diff2 = dX2 * dX2 + dY2 * dY2 + dZ2 * dZ2;
      float dis = c.x * c.x + c.y * c.y + c.z * c.z;
      if (D(diff) > 0.0002 * D(dis) && D(diff2) > 0.0002 * D(dis)) pk = 1;
    }
    // bit 1: the neighbour walk of :495-520 stops between i-1 and i
    int gap = 0;
    if (i >= 1) {
      const float4 a = sp[li], c = sp[li - 1];
      const float ex = a.x - c.x, ey = a.y - c.y, ez = a.z - c.z;
      gap = D(ex * ex + ey * ey + ez * ez) > 0.05 ? 1 : 0;
    }
    b.curv[gi] = cv;
    b.picked[gi] = (uint8_t)(pk | (gap << 1));
    // (sortInd = identity and labels 0 are implied: the selection's walk of dependent rings, the
    // one reader of the arrays, initialises them itself, sel_init)
  }
}

// ---------------------------------------------------------------- per-ring selection
template <int CAP, bool SIDX>
struct SelShared {
  uint64_t keys[CAP];       // (segment, curvature, position) of the ring; then (voxel, candidate)
  int sidx[SIDX ? CAP : 1]; // sortInd of the ring on entry (identity unless rings are walked in order)
  uint16_t cand[CAP];       // lessFlat candidate positions (relative to the ring start)
  uint8_t pk[CAP + 16];     // bit 0 cloudNeighborPicked, bit 1 neighbour-walk stop (gap)
  int8_t lab[CAP + 16];
  int se[128];
  int picks[kSharpPerRing + kLessSharpPerRing + kFlatPerRing];
  int scratch[16];
  float red[6][kSelThreads / 64];
  int order[64];
  int nsharp, nlsharp, nflat, ncand, wf, big, loff;
};

// dynamic LDS bytes added to each k_sr_ringvg workgroup (an occupancy cap for experiments)
#ifndef LOAM_RINGVG_PAD
#define LOAM_RINGVG_PAD 0
#endif
// member gathers in flight per step of a voxel's mean in ring_vg
#ifndef LOAM_VG_GATHER
#define LOAM_VG_GATHER 4  // (round 6: 8 -> 4, k_sr_select 1.34-1.35 -> 1.29 ms/step at 1024, 0.220 -> 0.215 at 128)
#endif
constexpr int kVgGather = LOAM_VG_GATHER;
#ifndef LOAM_RINGVG_HOLD
#define LOAM_RINGVG_HOLD 1
#endif
// PCL VoxelGrid 0.2 of one ring's lessFlat candidates pts[lo + cand[0..nc)) into
// outp (capacity outcap), the whole workgroup (:575-579): bbox, (voxel, candidate) keys, sort,
// ordered per-voxel float means.  Returns the voxel count (clamped to outcap, *err flagged).
template <int CAP, bool BIG, typename CandT>
LOAM_D int ring_vg(const float4* pts, int lo, const CandT* cand, int nc, uint64_t* keys, float4* outp, int outcap,
                   float (*red)[kSelThreads / 64], int* scratch, int* err) {
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
  // HOLD: the thread's candidates stay in registers from the bbox pass to the key pass (one read of
  // the candidates from memory instead of two)
  constexpr bool HOLD = !BIG && CAP <= 2048 && LOAM_RINGVG_HOLD;
  constexpr int RH = HOLD ? CAP / kSelThreads : 1;
  float4 held[RH];
  if constexpr (HOLD) {
#pragma unroll
    for (int e = 0; e < RH; ++e) {
      const int t = e * kSelThreads + tid;
      held[e] = t < nc ? pts[lo + cand[t]] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < RH; ++e)
      if (e * kSelThreads + tid < nc) {
        const float4 a = held[e];
        mn[0] = fminf(mn[0], a.x); mn[1] = fminf(mn[1], a.y); mn[2] = fminf(mn[2], a.z);
        mx[0] = fmaxf(mx[0], a.x); mx[1] = fmaxf(mx[1], a.y); mx[2] = fmaxf(mx[2], a.z);
      }
  } else {
    for (int t = tid; t < nc; t += kSelThreads) {
      const float4 a = pts[lo + cand[t]];
      mn[0] = fminf(mn[0], a.x); mn[1] = fminf(mn[1], a.y); mn[2] = fminf(mn[2], a.z);
      mx[0] = fmaxf(mx[0], a.x); mx[1] = fmaxf(mx[1], a.y); mx[2] = fmaxf(mx[2], a.z);
    }
  }
  for (int d = 0; d < 3; ++d) {
    mn[d] = wave_min_f_x(mn[d]);
    mx[d] = wave_max_f_x(mx[d]);
    if (lane == 0) { red[d][w] = mn[d]; red[3 + d][w] = mx[d]; }
  }
  __syncthreads();
  for (int d = 0; d < 3; ++d)
    for (int v = 0; v < kSelThreads / 64; ++v) {
      mn[d] = fminf(mn[d], red[d][v]);
      mx[d] = fmaxf(mx[d], red[3 + d][v]);
    }
  __syncthreads();
  int nout = 0;
  if (nc > 0) {
    const float inv = 1.0f / 0.2f;
    if (vg_leaf_too_small(mn, mx, inv)) {  // "leaf size too small": output = input
      for (int t = tid; t < nc; t += kSelThreads)
        if (t < outcap) outp[t] = pts[lo + cand[t]];
      nout = nc;
    } else {
      int minb[3], maxb[3];
      for (int d = 0; d < 3; ++d) {
        minb[d] = (int)floorf(mn[d] * inv);
        maxb[d] = (int)floorf(mx[d] * inv);
      }
      const int divx = maxb[0] - minb[0] + 1, divy = maxb[1] - minb[1] + 1;
      const int mul1 = divx, mul2 = divx * divy;
      if constexpr (!BIG) {
        // Candidates come in ring order, so consecutive ones mostly share a voxel (~2.2 per run on
        // VLP-16): sort the runs, (voxel, first candidate, length), instead of the candidates.
        // Runs of one voxel sorted by their first candidate list its members in the same order as
        // the stable (voxel, candidate) sort, so the means are summed in the same order.
        constexpr int NW = kSelThreads / 64;
        int nruns = 0;
        if constexpr (HOLD) {
          // all chunks at once: the thread's held candidates e * NT + tid, their run heads ranked by
          // wave ballots and the (chunk, wave) slots' counts prefixed in candidate order (two
          // barriers instead of four per chunk)
          static_assert(RH * NW <= 64, "slot prefix over one wave");
          __shared__ uint32_t rs_edge[RH * NW];
          __shared__ int rs_cnt[RH * NW];
          uint32_t idx[RH];
          int ex[RH];
#pragma unroll
          for (int e = 0; e < RH; ++e) {
            const int t = e * kSelThreads + tid;
            idx[e] = 0xffffffffu;
            if (t < nc) {
              const float4 a = held[e];
              const int i0 = (int)(floorf(a.x * inv) - (float)minb[0]);
              const int i1 = (int)(floorf(a.y * inv) - (float)minb[1]);
              const int i2 = (int)(floorf(a.z * inv) - (float)minb[2]);
              idx[e] = (uint32_t)(i0 + i1 * mul1 + i2 * mul2);
            }
            if (lane == 63) rs_edge[e * NW + w] = idx[e];
          }
          __syncthreads();
#pragma unroll
          for (int e = 0; e < RH; ++e) {
            const int t = e * kSelThreads + tid, slot = e * NW + w;
            uint32_t up = (uint32_t)__shfl_up((int)idx[e], 1, 64);
            if (lane == 0 && slot > 0) up = rs_edge[slot - 1];  // the previous 64 candidates' last
            const bool head = t < nc && (t == 0 || idx[e] != up);
            const uint64_t m = __ballot(head);
            ex[e] = head ? __popcll(m & lanemask_lt()) : -1;
            if (lane == 0) rs_cnt[slot] = __popcll(m);
          }
          __syncthreads();
          const int c = lane < RH * NW ? rs_cnt[lane] : 0;
          const int incl = wave_incl_scan_x(c);
          nruns = __shfl(incl, RH * NW - 1, 64);
#pragma unroll
          for (int e = 0; e < RH; ++e) {
            const int base = __shfl(incl - c, e * NW + w, 64);
            if (ex[e] >= 0) keys[base + ex[e]] = ((uint64_t)idx[e] << 32) | ((uint32_t)(e * kSelThreads + tid) << 16);
          }
        } else {
        uint32_t* edge = reinterpret_cast<uint32_t*>(&red[0][0]);  // last voxel of each wave's chunk
        for (int base = 0; base < nc; base += kSelThreads) {
          const int t = base + tid;
          uint32_t idx = 0xffffffffu;
          if (t < nc) {
            float4 a;
            if constexpr (HOLD) {
              a = held[0];
#pragma unroll
              for (int e = 1; e < RH; ++e)
                if (base == e * kSelThreads) a = held[e];
            } else {
              a = pts[lo + cand[t]];
            }
            const int i0 = (int)(floorf(a.x * inv) - (float)minb[0]);
            const int i1 = (int)(floorf(a.y * inv) - (float)minb[1]);
            const int i2 = (int)(floorf(a.z * inv) - (float)minb[2]);
            idx = (uint32_t)(i0 + i1 * mul1 + i2 * mul2);
          }
          uint32_t up = (uint32_t)__shfl_up((int)idx, 1, 64);
          if (lane == 63) edge[w + 1] = idx;
          __syncthreads();
          if (lane == 0) up = edge[w];  // edge[0]: the previous chunk's last candidate
          const int head = (t < nc && (t == 0 || idx != up)) ? 1 : 0;
          int tot;
          const int ex = block_excl_scan<kSelThreads>(head, scratch, tot);
          if (head) keys[nruns + ex] = ((uint64_t)idx << 32) | ((uint32_t)t << 16);
          if (tid == kSelThreads - 1) edge[0] = idx;
          nruns += tot;
        }
        }
        __syncthreads();
        constexpr int RE = CAP / kSelThreads;
        uint32_t nxt[RE];
#pragma unroll
        for (int e = 0; e < RE; ++e) {
          const int r = e * kSelThreads + tid;
          nxt[e] = r + 1 < nruns ? (uint32_t)keys[r + 1] >> 16 : (uint32_t)nc;
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < RE; ++e) {
          const int r = e * kSelThreads + tid;
          if (r < nruns) keys[r] |= nxt[e] - ((uint32_t)keys[r] >> 16);
        }
        __syncthreads();
        reg_bitonic_sort<kSelThreads, CAP / kSelThreads>(keys, nruns);
        // voxel heads among the sorted runs r = e * NT + tid, ranked like the runs above (one barrier)
        static_assert(RE * NW <= 64, "slot prefix over one wave");
        __shared__ int vs_cnt[RE * NW];
        int vex[RE];
#pragma unroll
        for (int e = 0; e < RE; ++e) {
          const int r = e * kSelThreads + tid;
          const bool head = r < nruns && (r == 0 || (keys[r] >> 32) != (keys[r - 1] >> 32));
          const uint64_t m = __ballot(head);
          vex[e] = head ? __popcll(m & lanemask_lt()) : -1;
          if (lane == 0) vs_cnt[e * NW + w] = __popcll(m);
        }
        __syncthreads();
        const int vc = lane < RE * NW ? vs_cnt[lane] : 0;
        const int vincl = wave_incl_scan_x(vc);
#pragma unroll
        for (int e = 0; e < RE; ++e) {
          const int r = e * kSelThreads + tid;
          const int vbase = __shfl(vincl - vc, e * NW + w, 64);
          if (vex[e] >= 0) {
            const int slot_out = vbase + vex[e];
            const uint32_t vk = (uint32_t)(keys[r] >> 32);
            float sx = 0, sy = 0, sz = 0, si = 0;
            int cnt = 0;
            // the voxel's members over all its runs (in run order, members ascending: the sorted
            // order), kVgGather gathers in flight per step whatever the run lengths
            int rr = r;
            uint32_t kk = (uint32_t)keys[r];
            int m = (int)(kk >> 16), m1 = m + (int)(kk & 0xffffu);
            const int mfirst = m;
            bool more = true;
            while (more) {
              int mi[kVgGather];
#pragma unroll
              for (int u = 0; u < kVgGather; ++u) {
                if (more && m >= m1) {  // the voxel's next run
                  ++rr;
                  if (rr < nruns && (uint32_t)(keys[rr] >> 32) == vk) {
                    kk = (uint32_t)keys[rr];
                    m = (int)(kk >> 16);
                    m1 = m + (int)(kk & 0xffffu);
                  } else {
                    more = false;
                  }
                }
                mi[u] = more ? m++ : -1;
              }
              float4 a[kVgGather];
#pragma unroll
              for (int u = 0; u < kVgGather; ++u) a[u] = pts[lo + cand[mi[u] >= 0 ? mi[u] : mfirst]];
#pragma unroll
              for (int u = 0; u < kVgGather; ++u)
                if (mi[u] >= 0) { sx += a[u].x; sy += a[u].y; sz += a[u].z; si += a[u].w; ++cnt; }
              if (more && m >= m1)  // run consumed: go on only when the voxel has another
                more = rr + 1 < nruns && (uint32_t)(keys[rr + 1] >> 32) == vk;
            }
            const float fc = (float)cnt;
            if (slot_out < outcap) outp[slot_out] = make_float4(sx / fc, sy / fc, sz / fc, si / fc);
          }
        }
        __syncthreads();  // the keys are read until here (a caller may reuse them)
        nout = __shfl(vincl, RE * NW - 1, 64);
      } else
      {
        const int P2c = next_pow2(nc);
        for (int t = tid; t < P2c; t += kSelThreads) {
          uint64_t key = ~0ull;
          if (t < nc) {
            const float4 a = pts[lo + cand[t]];
            int i0 = (int)(floorf(a.x * inv) - (float)minb[0]);
            int i1 = (int)(floorf(a.y * inv) - (float)minb[1]);
            int i2 = (int)(floorf(a.z * inv) - (float)minb[2]);
            uint32_t idx = (uint32_t)(i0 + i1 * mul1 + i2 * mul2);
            key = ((uint64_t)idx << 32) | (uint32_t)t;
          }
          keys[t] = key;
        }
        __syncthreads();
        if constexpr (BIG) block_bitonic_sort<kSelThreads>(keys, P2c);
        else reg_bitonic_sort<kSelThreads, CAP / kSelThreads>(keys, P2c);
        int run = 0;
        for (int base = 0; base < nc; base += kSelThreads) {
          const int t = base + tid;
          const int head = (t < nc && (t == 0 || (keys[t] >> 32) != (keys[t - 1] >> 32))) ? 1 : 0;
          int tot;
          const int ex = block_excl_scan<kSelThreads>(head, scratch, tot);
          if (head) {
            const uint32_t vk = (uint32_t)(keys[t] >> 32);
            int e = t + 1;
            while (e < nc && (uint32_t)(keys[e] >> 32) == vk) ++e;
            // members summed in sorted order; four independent gathers in flight per step
            float sx = 0, sy = 0, sz = 0, si = 0;
            for (int m = t; m < e; m += 4) {
              float4 a[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) a[u] = pts[lo + cand[(int)(keys[min(m + u, e - 1)] & 0xffffffffu)]];
#pragma unroll
              for (int u = 0; u < 4; ++u)
                if (m + u < e) { sx += a[u].x; sy += a[u].y; sz += a[u].z; si += a[u].w; }
            }
            const float cnt = (float)(e - t);
            if (run + ex < outcap) outp[run + ex] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
          }
          run += tot;
        }
        nout = run;
      }
    }
    if (nout > outcap) {
      if (tid == 0) atomicOr(err, ERR_CAP_RING);
      nout = outcap;
    }
  }
  return nout;
}

// :495-520 with the distance tests precomputed as gap bits.  One wave: lanes 0-4 take offsets
// +1..+5, lanes 8-12 offsets -1..-5; each direction marks up to its first stop (the reference's
// break), found with one ballot.  Every lane of the wave must call it (ind is wave-uniform).
LOAM_D void mark_neighbours(int n, int ind, uint8_t* pk, int wlo) {
  const int lane = lane_id();
  const bool pos = lane < 5, neg = lane >= 8 && lane < 13;
  const int off = pos ? lane + 1 : (neg ? 7 - lane : 0);
  bool stop = false;
  if (pos) stop = ind + off >= n || (pk[ind + off - wlo] & 2);
  else if (neg) stop = ind + off < 0 || (pk[ind + off + 1 - wlo] & 2);
  const uint64_t sm = __ballot(stop);
  const uint64_t sp = sm & 0x1full, sn = (sm >> 8) & 0x1full;
  const int np = sp ? __ffsll((unsigned long long)sp) - 1 : 5;   // offsets marked in each direction
  const int nn = sn ? __ffsll((unsigned long long)sn) - 1 : 5;
  if ((pos && lane < np) || (neg && lane - 8 < nn)) pk[ind + off - wlo] |= 1;
}

// The greedy picks of one segment [sp, ep] (ring-local) for independent rings (one wave):
// :476-522 sharp / less sharp and :524-566 flat, on the ring's curvatures cv and the LDS pick state.
// SR > 0: the segment is at most 64 * SR points and its curvatures are read once into SR registers
// per lane (the flat walk rescans them up to four times).
// crin: the caller's registers with cv[sp + 64 k + lane] (loaded ahead, during the previous segment).
// pre(): called once the compaction has consumed crin (the caller issues its next loads there).
struct NoPre {
  LOAM_D void operator()() const {}
};
template <int SR = 0, typename Pre = NoPre>
LOAM_D void select_segment_fast(int n, int lo, int sp, int ep, const float* cv, uint64_t* list, uint8_t* pk,
                                int8_t* lab, int wlo, int* picks, int& nsharp, int& nlsharp, int& nflat,
                                const float* crin = nullptr, Pre pre = Pre()) {
  const int lane = lane_id();
  float cr[SR > 0 ? SR : 1];
  if constexpr (SR > 0) {
#pragma unroll
    for (int k = 0; k < SR; ++k) cr[k] = crin[k];
  }
  if constexpr (SR > 0) {
    // The sharp walk (:476-522) takes the points with curvature > 0.1 from the top of the stable
    // ascending sort: by (curvature, position) descending, skipping a marked point, until the 21st
    // pick.  Marks only grow, so its next pick is always the largest (curvature bits, position) key
    // among the unmarked candidates: repeated wave arg-max over the segment's register-held
    // curvatures, no sort (the flat pass below is the same walk from the bottom).
    pre();
    int largest = 0;
    for (;;) {
      uint64_t nkey = ~0ull;  // complemented keys: the minimum is the largest key
#pragma unroll
      for (int k = 0; k < SR; ++k) {
        const int t = sp + k * 64 + lane;
        if (t <= ep && D(cr[k]) > 0.1 && (pk[lo + t - wlo] & 1) == 0) {
          const uint64_t key = ~(((uint64_t)fkey(cr[k]) << 32) | (uint32_t)t);
          nkey = key < nkey ? key : nkey;
        }
      }
      nkey = wave_min_u64_x(nkey);
      if (nkey == ~0ull) break;
      largest++;
      if (largest > 20) break;
      const int ind = lo + (int)(uint32_t)~nkey;
      if (lane == 0) {
        if (largest <= 2) {
          lab[ind - wlo] = 2;
          picks[nsharp++] = ind;
          picks[kSharpPerRing + nlsharp++] = ind;
        } else {
          lab[ind - wlo] = 1;
          picks[kSharpPerRing + nlsharp++] = ind;
        }
        pk[ind - wlo] |= 1;
      }
      mark_neighbours(n, ind, pk, wlo);
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
    }
  }
  // points with curvature > 0.1, as (curvature bits, position): ascending = the stable sort's order
  int m = 0;
  if constexpr (SR > 0) {
  } else {
    for (int base = sp; base <= ep; base += 64) {
      const int t = base + lane;
      const bool e = t <= ep && D(cv[t]) > 0.1;
      const uint64_t bm = __ballot(e);
      if (e) list[m + __popcll(bm & lanemask_lt())] = ((uint64_t)fkey(cv[t]) << 32) | (uint32_t)t;
      m += __popcll(bm);
    }
  }
  if constexpr (SR == 0) pre();
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  if (SR == 0 && m > 1) wave_sort_u64(list, m);
  int largest = 0;
  bool done = false;
  for (int base = m - 1; SR == 0 && base >= 0 && !done; base -= 64) {  // from the largest curvature down
    const int k = base - lane;
    const bool elig = k >= 0;
    const int ind = elig ? lo + (int)(uint32_t)list[k] : 0;
    uint64_t remaining = __ballot(elig);
    while (remaining) {
      const bool cand_ok = elig && ((remaining >> lane) & 1ull) && (pk[ind - wlo] & 1) == 0;
      const uint64_t mm = __ballot(cand_ok);
      if (!mm) break;
      const int f = __ffsll((unsigned long long)mm) - 1;
      largest++;
      if (largest > 20) { done = true; break; }
      if (lane == f) {
        if (largest <= 2) {
          lab[ind - wlo] = 2;
          picks[nsharp++] = ind;
          picks[kSharpPerRing + nlsharp++] = ind;
        } else {
          lab[ind - wlo] = 1;
          picks[kSharpPerRing + nlsharp++] = ind;
        }
        pk[ind - wlo] |= 1;
      }
      mark_neighbours(n, __builtin_amdgcn_readlane(ind, f), pk, wlo);
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
      remaining &= ~((2ull << f) - 1ull);
    }
  }
  // flat: the unmarked point of smallest (curvature, position) below 0.1, four times at most
  for (int smallest = 0;;) {
    uint64_t best = ~0ull;
    if constexpr (SR > 0) {
#pragma unroll
      for (int k = 0; k < SR; ++k) {
        const int t = sp + k * 64 + lane;
        if (t <= ep && D(cr[k]) < 0.1 && (pk[lo + t - wlo] & 1) == 0) {
          const uint64_t key = ((uint64_t)fkey(cr[k]) << 32) | (uint32_t)t;
          best = key < best ? key : best;
        }
      }
    } else {
      for (int t = sp + lane; t <= ep; t += 64) {
        const float c = cv[t];
        if (D(c) < 0.1 && (pk[lo + t - wlo] & 1) == 0) {
          const uint64_t key = ((uint64_t)fkey(c) << 32) | (uint32_t)t;
          best = key < best ? key : best;
        }
      }
    }
    best = wave_min_u64_x(best);
    if (best == ~0ull) break;
    const int ind = lo + (int)(uint32_t)best;
    if (lane == 0) {
      lab[ind - wlo] = -1;
      picks[kSharpPerRing + kLessSharpPerRing + nflat++] = ind;
    }
    if (++smallest >= 4) break;  // after the push, before the marks (:555-557)
    if (lane == 0) pk[ind - wlo] |= 1;
    mark_neighbours(n, ind, pk, wlo);
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
  }
}

// ring sort key: segment (3 bits) | curvature bits (32) | position in the ring (29)
constexpr int kPosBits = 29;
constexpr uint64_t kPosMask = (1ull << kPosBits) - 1;
LOAM_D float key_curv(uint64_t key) { return __builtin_bit_cast(float, (uint32_t)(key >> kPosBits)); }

// processes ring q of sweep s; `seq` = rings walked in order by one workgroup (dependent rings).
// The six segment sorts (:466-474) are one sort of the ring by (segment, curvature, position):
// the segments partition the ring span and the sort does not depend on the picks.  The greedy
// picks and the lessFlat candidates of each segment are then one wave's work.
// CAP: LDS capacity of the ring state.  BIG: the ring state lives in global scratch (slot `slot`)
// and in the sweep's own picked / label arrays, for spans beyond any LDS capacity (an empty ring
// leaves its successor spanning every earlier ring, Q5).
// SIDX: the ring's sortInd may differ from the identity (rings walked in order); without it the
// ring state holds no sortInd copy (8 KB less LDS) and sortInd[k] = k.
template <int CAP, bool BIG, bool SIDX>
LOAM_D void select_ring(const SrBuffers& b, int s, int q, int R, int n, bool seq, SelShared<CAP, SIDX>& sh, int slot) {
  using CandT = typename std::conditional<BIG, int, uint16_t>::type;
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const float4* pts = b.full + (size_t)s * b.cap;
  const float* curv = b.curv + (size_t)s * b.cap;
  const int sq = sh.se[q], eq = sh.se[R + q];
  const int lo = sq, hi = eq - 1;
  const int loff = BIG ? sh.loff : q * kRingCap;   // lessFlat staging offset of this ring
  if (tid == 0) { sh.nsharp = 0; sh.nlsharp = 0; sh.nflat = 0; sh.ncand = 0; }
  int* st_cnt = b.st_cnt + (size_t)(s * R + q) * 4;
  if (tid == 0) b.st_loff[s * R + q] = loff;
  if (lo > hi) {  // every segment is empty
    if (tid < 4) st_cnt[tid] = 0;
    return;
  }
  if ((!BIG && hi - lo + 1 > CAP) || lo < 0 || hi >= n) {
    if (tid == 0) b.err[s] |= ERR_CAP_RING;
    if (tid < 4) st_cnt[tid] = 0;
    return;
  }
  const int len = hi - lo + 1;
  // window of point indices this ring may touch: span and the indices its sortInd holds, +-5
  int vmin = lo, vmax = hi;
  if (seq && !BIG) {
    for (int k = lo + tid; k <= hi; k += kSelThreads) {
      int v = b.sortind[(size_t)s * b.cap + k];
      vmin = min(vmin, v);
      vmax = max(vmax, v);
    }
    vmin = wave_min_i(vmin);
    vmax = wave_max_i(vmax);
    if (lane == 0) { sh.scratch[w] = vmin; sh.scratch[8 + w] = vmax; }
    __syncthreads();
    for (int v = 0; v < kSelThreads / 64; ++v) {
      vmin = min(vmin, sh.scratch[v]);
      vmax = max(vmax, sh.scratch[8 + v]);
    }
    __syncthreads();
  }
  const int wlo = BIG ? 0 : max(0, vmin - 5), whi = BIG ? n - 1 : min(n - 1, vmax + 5);
  if (!BIG && whi - wlo + 1 > CAP + 16) {
    if (tid == 0) b.err[s] |= ERR_CAP_RING;
    if (tid < 4) st_cnt[tid] = 0;
    return;
  }
  uint64_t* keys;
  int* sidx;
  CandT* cand;
  uint8_t* pk;
  int8_t* lab;
  if constexpr (BIG) {
    const size_t so = (size_t)slot * b.big_stride;
    keys = b.big_keys + so;
    sidx = b.big_sidx + so;
    cand = b.big_cand + so;
    pk = b.picked + (size_t)s * b.cap;
    lab = b.label + (size_t)s * b.cap;
  } else {
    keys = sh.keys;
    sidx = SIDX ? sh.sidx : nullptr;
    cand = sh.cand;
    pk = sh.pk;
    lab = sh.lab;
    for (int k = wlo + tid; k <= whi; k += kSelThreads) {
      pk[k - wlo] = b.picked[(size_t)s * b.cap + k];
      lab[k - wlo] = SIDX && seq ? b.label[(size_t)s * b.cap + k] : 0;  // labels start at 0 (sel_init)
    }
  }
  int segb[7];
#pragma unroll
  for (int j = 0; j <= 6; ++j) segb[j] = (sq * (6 - j) + eq * j) / 6;  // sp_j; ep_j = sp_{j+1} - 1
  // FAST (independent rings, sortInd = identity): no ring sort.  The sharp walk visits only the
  // points with curvature > 0.1, so those are compacted and sorted per segment (one wave, in
  // registers); the flat walk stops at its 4th pick, so it is a repeated minimum over the eligible
  // points (an arg-min over "unmarked and < 0.1" is the next point the ascending walk would take:
  // marks only accumulate).  cv: the ring's curvatures in the upper half of keys.
  constexpr bool FAST = !SIDX && !BIG;
  float* cv = reinterpret_cast<float*>(keys + CAP / 2);
  if constexpr (FAST) {
    for (int t = tid; t < len; t += kSelThreads) cv[t] = curv[lo + t];
    __syncthreads();
  } else {
  const int P2 = next_pow2(len);
  for (int t = tid; t < P2; t += kSelThreads) {
    uint64_t key = ~0ull;
    if (t < len) {
      const int v = SIDX && seq ? b.sortind[(size_t)s * b.cap + lo + t] : lo + t;
      if (SIDX) sidx[t] = v;
      int seg = 0;
#pragma unroll
      for (int j = 1; j < 6; ++j) seg += (lo + t >= segb[j]) ? 1 : 0;
      key = ((uint64_t)seg << 61) | ((uint64_t)fkey(curv[v]) << kPosBits) | (uint64_t)t;
    }
    keys[t] = key;
  }
  __syncthreads();
  if constexpr (BIG) block_bitonic_sort<kSelThreads>(keys, P2);
  else reg_bitonic_sort<kSelThreads, CAP / kSelThreads>(keys, P2);
  }
  if (w == 0) {
    int run = 0;
    for (int j = 0; j < 6; ++j) {
      const int sp = segb[j] - lo, ep = segb[j + 1] - 1 - lo;  // sorted-local range of segment j
      if (ep < sp) continue;
      if constexpr (FAST) {
        select_segment_fast(n, lo, sp, ep, cv, keys, pk, lab, wlo, sh.picks, sh.nsharp, sh.nlsharp, sh.nflat);
      } else {
      // (:476-522) sharp / less sharp, walking from the largest curvature down
      int largest = 0;
      bool done = false;
      for (int base = ep; base >= sp && !done; base -= 64) {
        const int k = base - lane;
        const bool inr = k >= sp;
        const uint64_t key = inr ? keys[k] : 0ull;
        const int ind = inr ? (SIDX ? sidx[key & kPosMask] : lo + (int)(key & kPosMask)) : 0;
        const bool elig = inr && D(key_curv(key)) > 0.1;
        uint64_t remaining = __ballot(elig);
        if (remaining != __ballot(inr)) done = true;  // sorted: no eligible point below this chunk
        while (remaining) {
          const bool cand_ok = elig && ((remaining >> lane) & 1ull) && (pk[ind - wlo] & 1) == 0;
          const uint64_t m = __ballot(cand_ok);
          if (!m) break;
          const int f = __ffsll((unsigned long long)m) - 1;
          largest++;
          if (largest > 20) { done = true; break; }
          if (lane == f) {
            if (largest <= 2) {
              lab[ind - wlo] = 2;
              sh.picks[sh.nsharp++] = ind;
              sh.picks[kSharpPerRing + sh.nlsharp++] = ind;
            } else {
              lab[ind - wlo] = 1;
              sh.picks[kSharpPerRing + sh.nlsharp++] = ind;
            }
            pk[ind - wlo] |= 1;
          }
          mark_neighbours(n, __builtin_amdgcn_readlane(ind, f), pk, wlo);
          __threadfence_block();
          __builtin_amdgcn_wave_barrier();
          remaining &= ~((2ull << f) - 1ull);
        }
      }
      // (:524-566) flat, walking from the smallest curvature up; break after the 4th push
      int smallest = 0;
      done = false;
      for (int base = sp; base <= ep && !done; base += 64) {
        const int k = base + lane;
        const bool inr = k <= ep;
        const uint64_t key = inr ? keys[k] : 0ull;
        const int ind = inr ? (SIDX ? sidx[key & kPosMask] : lo + (int)(key & kPosMask)) : 0;
        const bool elig = inr && D(key_curv(key)) < 0.1;
        uint64_t remaining = __ballot(elig);
        const bool last = remaining != __ballot(inr);  // sorted: no eligible point above this chunk
        while (remaining) {
          const bool cand_ok = elig && ((remaining >> lane) & 1ull) && (pk[ind - wlo] & 1) == 0;
          const uint64_t m = __ballot(cand_ok);
          if (!m) break;
          const int f = __ffsll((unsigned long long)m) - 1;
          if (lane == f) {
            lab[ind - wlo] = -1;
            sh.picks[kSharpPerRing + kLessSharpPerRing + sh.nflat++] = ind;
          }
          smallest++;
          if (smallest >= 4) { done = true; break; }
          if (lane == f) pk[ind - wlo] |= 1;
          mark_neighbours(n, __builtin_amdgcn_readlane(ind, f), pk, wlo);
          __threadfence_block();
          __builtin_amdgcn_wave_barrier();
          remaining &= ~((2ull << f) - 1ull);
        }
        if (last) done = true;
      }
      }  // !FAST
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
      // (:568-572) lessFlat candidates of this segment, in position order
      for (int base = segb[j]; base < segb[j + 1]; base += 64) {
        const int k = base + lane;
        const bool flag = k < segb[j + 1] && lab[k - wlo] <= 0;
        const uint64_t m = __ballot(flag);
        if (flag) cand[run + __popcll(m & lanemask_lt())] = (CandT)(k - lo);
        run += __popcll(m);
      }
    }
    if (lane == 0) sh.ncand = run;
  }
  __syncthreads();
  if (SIDX && seq) {  // the ring's sortInd after its six sorts, for the next ring (one workgroup, ordered)
    for (int t = tid; t < len; t += kSelThreads)
      b.sortind[(size_t)s * b.cap + lo + t] = sidx[keys[t] & kPosMask];
    __syncthreads();
  }
  // ---- PCL VoxelGrid 0.2 of the ring's lessFlat candidates (:575-579)
  const int nout = ring_vg<CAP, BIG>(pts, lo, cand, sh.ncand, keys, b.st_lflat + (size_t)s * R * kRingCap + loff,
                                     BIG ? R * kRingCap - loff : kRingCap, sh.red, sh.scratch, b.err + s);
  // pick lists -> staging
  const int ns = sh.nsharp, nl = sh.nlsharp, nf = sh.nflat;
  for (int t = tid; t < ns; t += kSelThreads) b.st_sharp[(size_t)(s * R + q) * kSharpPerRing + t] = sh.picks[t];
  for (int t = tid; t < nl; t += kSelThreads)
    b.st_lsharp[(size_t)(s * R + q) * kLessSharpPerRing + t] = sh.picks[kSharpPerRing + t];
  for (int t = tid; t < nf; t += kSelThreads)
    b.st_flat[(size_t)(s * R + q) * kFlatPerRing + t] = sh.picks[kSharpPerRing + kLessSharpPerRing + t];
  if (tid == 0) { st_cnt[0] = ns; st_cnt[1] = nl; st_cnt[2] = nf; st_cnt[3] = nout; }
  if (BIG && tid == 0) sh.loff = loff + nout;
  if (seq && !BIG) {  // write the shared state back for the next ring (one workgroup, ordered)
    for (int k = wlo + tid; k <= whi; k += kSelThreads) {
      b.picked[(size_t)s * b.cap + k] = pk[k - wlo];
      b.label[(size_t)s * b.cap + k] = lab[k - wlo];
    }
  }
  __threadfence();
  __syncthreads();
}

// ---------------------------------------------------------------- selection split: picks / VoxelGrid
// Sweeps whose rings are independent and at most kPickCap points long (every VLP-16 / HDL-64E
// sweep without an empty ring) take two kernels instead of k_sr_select<2048, 0>:
//  k_sr_pick    one WAVE per ring (kPickWaves rings per workgroup): the greedy sharp / flat picks
//               of the six segments (select_segment_fast, wave-synchronous, no workgroup barrier)
//               and the ring's lessFlat candidate list, to global memory;
//  k_sr_ringvg  one workgroup per ring: the PCL VoxelGrid of the candidates (ring_vg).
// The serial greedy walk no longer holds three idle waves of a workgroup at barriers, and the
// VoxelGrid runs at full workgroup occupancy.  Other sweeps fall to k_sr_select<4096, 1> / <16, 2>
// exactly as before (sel_big).
constexpr int kPickCap = 2048;
constexpr int kSelListGrid = 32;  // k_sr_select<4096, 1> workgroup rows over its listed sweeps
// rings (waves) per k_sr_pick workgroup: one, so a workgroup's LDS is freed as soon as its own ring's
// greedy walk ends (k_sr_select ms/step at batch 1024: 4 -> 1.67-1.69, 2 -> 1.66, 1 -> 1.63-1.65)
constexpr int kPickWaves = 1;
constexpr int kPickWpe = 4;  // <= 128 VGPRs: four waves per SIMD (the LDS allows four workgroups per CU)
constexpr int kPickSegRegs = (kPickCap / 6 + 2 + 63) / 64;  // a segment of a <= kPickCap ring, per lane

struct PickWave {  // (no candidate list: the register path's picks are wave arg-maxes)
  uint8_t pk[kPickCap + 16];
  int8_t lab[kPickCap + 16];
  int picks[kSharpPerRing + kLessSharpPerRing + kFlatPerRing];
  int nsharp, nlsharp, nflat;
};

// the sweep's ring bounds (:392-393 fix-ups) into se[0..2R), and the selection route of the sweep
// (0: rings independent and <= cap points, 1: k_sr_select<4096, 1>), valid in thread 0.  Wave 0
// evaluates the ordered walk below with a lane per ring: each active ring's predecessor in the
// (start, ring) order is found by a max over the other lanes (no serial insertion sort).
LOAM_D int sweep_route(const SrBuffers& b, int s, int R, int n, int cap, int* se, int* order) {
  const int tid = threadIdx.x;
  if (tid < R) {
    int st = b.ring_se[s * 2 * R + tid], en = b.ring_se[s * 2 * R + R + tid];
    if (tid == 0) st = 5;
    if (tid == R - 1) en = n - 5;
    se[tid] = st;
    se[R + tid] = en;
  }
  __syncthreads();
  int next = 0;
  (void)order;
  if (tid < 64) {  // R <= 64
    const int r = tid;
    const bool act = r < R && se[r] <= se[R + r] - 1;
    const int lo = act ? se[r] : 0, hi = act ? se[R + r] - 1 : 0;
    const uint64_t am = __ballot(act);
    // predecessor of r in the insertion sort's order (start ascending, ring index on ties)
    int pst = 0, pidx = -1, phi = -100000;  // -100000: the walk's initial prev_hi
    for (int k = 0; k < R; ++k) {
      const int ks = __builtin_amdgcn_readlane(lo, k), kh = __builtin_amdgcn_readlane(hi, k);
      const bool before = (ks < lo || (ks == lo && k < r));
      if (((am >> k) & 1) && before && (pidx < 0 || ks > pst || (ks == pst && k > pidx))) {
        pst = ks;
        pidx = k;
        phi = kh;
      }
    }
    const bool fail = act && (lo < 0 || hi >= n || lo - phi <= 5);
    const int maxspan = wave_max_i(act ? hi - lo + 1 : 0);
    const bool wf = __ballot(fail) == 0;
    if (n > 0 && (!wf || maxspan > cap)) next = 1;
  }
  return next;
}

__global__ __launch_bounds__(64 * kPickWaves) __attribute__((amdgpu_waves_per_eu(kPickWpe))) void k_sr_pick(SrBuffers b, SrParams p) {
  const int s = blockIdx.y, tid = threadIdx.x, w = tid >> 6, lane = lane_id(), R = p.R;
  const int q = blockIdx.x * kPickWaves + w;
  __shared__ int se[128], order[64], sh_route;
  __shared__ PickWave pw[kPickWaves];
  const int n = b.n_full[s];
  const int route = sweep_route(b, s, R, n, kPickCap, se, order);
  if (tid == 0) {
    sh_route = route;
    if (blockIdx.x == 0) {
      b.sel_big[s] = route;
      if (route) b.sel_list[2 + atomicAdd(&b.sel_list[0], 1)] = s;  // (k_sr_select<4096, 1>'s sweeps)
    }
  }
  __syncthreads();
  if (sh_route != 0 || q >= R) return;  // wave-uniform from here on: no workgroup barrier below
  PickWave& P = pw[w];
  int* st_cnt = b.st_cnt + (size_t)(s * R + q) * 4;
  if (lane == 0) b.st_loff[s * R + q] = q * kRingCap;
  const int sq = se[q], eq = se[R + q];
  const int lo = sq, hi = eq - 1;
  if (n <= 0 || lo > hi || hi - lo + 1 > kPickCap || lo < 0 || hi >= n) {
    if (n > 0 && lo <= hi && lane == 0) atomicOr(&b.err[s], ERR_CAP_RING);
    if (lane < 4) st_cnt[lane] = 0;
    if (lane == 0) b.st_ncand[s * R + q] = 0;
    return;
  }
  const int wlo = max(0, lo - 5), whi = min(n - 1, hi + 5);
  const uint8_t* pick_g = b.picked + (size_t)s * b.cap;
  for (int k = wlo + lane; k <= whi; k += 64) {
    P.pk[k - wlo] = pick_g[k];
    P.lab[k - wlo] = 0;
  }
  if (lane == 0) { P.nsharp = 0; P.nlsharp = 0; P.nflat = 0; }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  const float* cv = b.curv + (size_t)s * b.cap + lo;
  uint16_t* cand = b.st_cand + (size_t)(s * R + q) * kRingCap;
  int run = 0;
  // each segment's curvatures are loaded while the previous segment is walked
  float cra[kPickSegRegs], crb[kPickSegRegs];
  auto load_seg = [&](int j, float* cr) {
    const int s0 = (sq * (6 - j) + eq * j) / 6, s1 = (sq * (5 - j) + eq * (j + 1)) / 6;
#pragma unroll
    for (int k = 0; k < kPickSegRegs; ++k) {
      const int t = s0 - lo + k * 64 + lane;
      cr[k] = t <= s1 - 1 - lo ? cv[t] : 0.0f;
    }
  };
  load_seg(0, cra);
  for (int j = 0; j < 6; ++j) {
    const int s0 = (sq * (6 - j) + eq * j) / 6, s1 = (sq * (5 - j) + eq * (j + 1)) / 6;  // sp_j, ep_j + 1
    auto pre = [&]() {
      if (j < 5) load_seg(j + 1, crb);
    };
    if (s1 - 1 < s0) pre();
    if (s1 - 1 >= s0) {
    select_segment_fast<kPickSegRegs>(n, lo, s0 - lo, s1 - 1 - lo, cv, nullptr, P.pk, P.lab, wlo, P.picks, P.nsharp,
                                      P.nlsharp, P.nflat, cra, pre);
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    // (:568-572) lessFlat candidates of this segment, in position order
    for (int base = s0; base < s1; base += 64) {
      const int k = base + lane;
      const bool flag = k < s1 && P.lab[k - wlo] <= 0;
      const uint64_t m = __ballot(flag);
      if (flag) cand[run + __popcll(m & lanemask_lt())] = (uint16_t)(k - lo);
      run += __popcll(m);
    }
    }
#pragma unroll
    for (int k = 0; k < kPickSegRegs; ++k) cra[k] = crb[k];
  }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  const int ns = P.nsharp, nl = P.nlsharp, nf = P.nflat;
  for (int t = lane; t < ns; t += 64) b.st_sharp[(size_t)(s * R + q) * kSharpPerRing + t] = P.picks[t];
  for (int t = lane; t < nl; t += 64) b.st_lsharp[(size_t)(s * R + q) * kLessSharpPerRing + t] = P.picks[kSharpPerRing + t];
  for (int t = lane; t < nf; t += 64)
    b.st_flat[(size_t)(s * R + q) * kFlatPerRing + t] = P.picks[kSharpPerRing + kLessSharpPerRing + t];
  if (lane == 0) { st_cnt[0] = ns; st_cnt[1] = nl; st_cnt[2] = nf; b.st_ncand[s * R + q] = run; }
}

__global__ __launch_bounds__(kSelThreads) void k_sr_ringvg(SrBuffers b, SrParams p) {
  const int q = blockIdx.x, s = blockIdx.y, tid = threadIdx.x, R = p.R;
  // the ring's words loaded together (one round trip), then the early exits
  const int big = b.sel_big[s], n = b.n_full[s];
  int lo = b.ring_se[s * 2 * R + q], en = b.ring_se[s * 2 * R + R + q];
  const int nc = min(b.st_ncand[s * R + q], kPickCap);
  if (big != 0 || n <= 0) return;
  if (q == 0) lo = 5;
  if (q == R - 1) en = n - 5;
  if (lo > en - 1) return;
  __shared__ uint64_t keys[kPickCap];
  __shared__ uint16_t cand[kPickCap];
  __shared__ float red[6][kSelThreads / 64];
  __shared__ int scratch[16];
  const uint16_t* cg = b.st_cand + (size_t)(s * R + q) * kRingCap;
  for (int t = tid; t < nc; t += kSelThreads) cand[t] = cg[t];
  __syncthreads();
  const int nout = ring_vg<kPickCap, false>(b.full + (size_t)s * b.cap, lo, cand, nc, keys,
                                            b.st_lflat + (size_t)s * R * kRingCap + q * kRingCap, kRingCap, red,
                                            scratch, b.err + s);
  if (tid == 0) b.st_cnt[(size_t)(s * R + q) * 4 + 3] = nout;
}

// sortInd = identity and labels 0 over sweep s (the workgroup), before a walk of dependent rings
// reads and writes them back ring by ring (k_sr_features leaves them unwritten: the common path,
// independent rings, never reads them)
LOAM_D void sel_init(const SrBuffers& b, int s, int n) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    b.sortind[(size_t)s * b.cap + k] = k;
    b.label[(size_t)s * b.cap + k] = 0;
  }
  __threadfence_block();
  __syncthreads();
}

// Three instantiations, chosen per sweep: CAP = 2048 (34 KB of LDS, four workgroups per CU)
// takes every sweep whose rings are independent and no longer than 2048 points (VLP-16,
// HDL-64E) and flags the others (sel_big = 1); CAP = 4096 redoes those whose spans fit it, rings
// walked in order when they depend on each other, and flags the rest (sel_big = 2); the global-
// memory variant walks those (gridDim.x workgroups over the flagged sweeps, one scratch slot each).
template <int CAP, int MODE>  // MODE 0: fast, 1: 4096 / dependent rings, 2: unbounded spans
__global__ __launch_bounds__(kSelThreads) __attribute__((amdgpu_waves_per_eu(MODE == 0 ? 6 : 1))) void k_sr_select(SrBuffers b, SrParams p) {
  constexpr bool BIG = MODE == 2;
  const int tid = threadIdx.x, R = p.R;
  constexpr bool SIDX = MODE != 0;  // MODE 0 takes independent rings only
  __shared__ SelShared<CAP, SIDX> sh;
  // MODE 1 / 2: the sweeps k_sr_pick / MODE 1 routed here (sel_list), gridDim.y / gridDim.x workgroups
  // (of R rings / one) over them; MODE 0: sweep blockIdx.y
  const int nlist = MODE == 0 ? b.S : b.sel_list[MODE - 1];
  const int* list = b.sel_list + 2 + (MODE == 2 ? b.S : 0);
  for (int i = BIG ? blockIdx.x : blockIdx.y; i < nlist; i += BIG ? gridDim.x : gridDim.y) {
    const int s = MODE == 0 ? i : list[i];
    const int q = BIG ? 0 : blockIdx.x;
    if (MODE != 0 && b.sel_big[s] != MODE) continue;
    const int n = b.n_full[s];
    if (tid < R) {
      int st = b.ring_se[s * 2 * R + tid], en = b.ring_se[s * 2 * R + R + tid];
      if (tid == 0) st = 5;            // :392
      if (tid == R - 1) en = n - 5;    // :393
      sh.se[tid] = st;
      sh.se[R + tid] = en;
    }
    __syncthreads();
    if (tid == 0) {
      // rings are independent when their active spans [start, end-1] are more than 5 points apart
      int wf = 1, prev_hi = -100000, maxspan = 0;
      int* order = sh.order;
      int na = 0;
      for (int r = 0; r < R; ++r)
        if (sh.se[r] <= sh.se[R + r] - 1) order[na++] = r;
      for (int a = 1; a < na; ++a) {
        int v = order[a], c = a;
        while (c > 0 && sh.se[order[c - 1]] > sh.se[v]) { order[c] = order[c - 1]; --c; }
        order[c] = v;
      }
      for (int a = 0; a < na; ++a) {
        int lo = sh.se[order[a]], hi = sh.se[R + order[a]] - 1;
        if (lo < 0 || hi >= n || lo - prev_hi <= 5) wf = 0;
        maxspan = max(maxspan, hi - lo + 1);
        prev_hi = hi;
      }
      sh.wf = wf;
      sh.loff = 0;
      int next = MODE;
      if (MODE == 0 && n > 0 && (!wf || maxspan > CAP)) next = 1;
      if (MODE == 1 && n > 0 && maxspan > CAP) next = 2;
      sh.big = next != MODE;
      if (q == 0 && MODE != 2) {
        b.sel_big[s] = next;
        if (MODE == 1 && next == 2) b.sel_list[2 + b.S + atomicAdd(&b.sel_list[1], 1)] = s;
      }
    }
    __syncthreads();
    if (!sh.big) {
      if (n <= 0) {
        if (tid < 4) b.st_cnt[(size_t)(s * R + q) * 4 + tid] = 0;
        if (tid == 0) b.st_loff[s * R + q] = q * kRingCap;
      } else if (sh.wf && !BIG) {
        select_ring<CAP, BIG, SIDX>(b, s, q, R, n, false, sh, 0);
      } else if (q == 0) {
        if constexpr (SIDX) {
          sel_init(b, s, n);
          for (int r = 0; r < R; ++r) select_ring<CAP, BIG, SIDX>(b, s, r, R, n, true, sh, BIG ? blockIdx.x : 0);
        }
      }
    }
    __syncthreads();
    if (MODE == 0) break;
  }
}

// ---------------------------------------------------------------- compaction
__global__ __launch_bounds__(256) void k_sr_compact(SrBuffers b, SrParams p) {
  // one workgroup per (ring, sweep): the ring's offsets are the counts of the rings before it
  const int r = blockIdx.x, s = blockIdx.y, tid = threadIdx.x, R = p.R;
  __shared__ int off[4];
  if (tid < 4) {
    int run = 0, all = 0;
    for (int q = 0; q < R; ++q) {
      const int c = b.st_cnt[(size_t)(s * R + q) * 4 + tid];
      run += q < r ? c : 0;
      all += c;
    }
    off[tid] = run;
    if (r == 0) b.cnt[s * 4 + tid] = all;
  }
  __syncthreads();
  const float4* pts = b.full + (size_t)s * b.cap;
  const int* c = b.st_cnt + (size_t)(s * R + r) * 4;
  const int c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
  for (int t = tid; t < c0; t += 256)
    b.sharp[(size_t)s * kSharpPerRing * R + off[0] + t] = pts[b.st_sharp[(size_t)(s * R + r) * kSharpPerRing + t]];
  for (int t = tid; t < c1; t += 256)
    b.lsharp[(size_t)s * kLessSharpPerRing * R + off[1] + t] =
        pts[b.st_lsharp[(size_t)(s * R + r) * kLessSharpPerRing + t]];
  for (int t = tid; t < c2; t += 256)
    b.flat[(size_t)s * kFlatPerRing * R + off[2] + t] = pts[b.st_flat[(size_t)(s * R + r) * kFlatPerRing + t]];
  const float4* lf = b.st_lflat + (size_t)s * R * kRingCap + b.st_loff[s * R + r];
  for (int t = tid; t < c3; t += 256) b.lflat[(size_t)s * b.cap + off[3] + t] = lf[t];
}

}  // namespace

#define HIPCHK(x) (void)(x)

__global__ __launch_bounds__(256) void k_sr_scatter_packed(const float4* src, const int* off, const int* n, float4* raw,
                                                         int cap) {
  const int s = blockIdx.y, m = n[s], o = off[s];
  for (int t = blockIdx.x * 256 + threadIdx.x; t < m; t += gridDim.x * 256) raw[(size_t)s * cap + t] = src[(size_t)o + t];
}

hipError_t sr_scatter_packed(const float4* src, const int* off, const int* n, float4* raw, int cap, int S,
                             hipStream_t st) {
  if (S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_sr_scatter_packed, dim3(std::max(1, std::min(64, (cap + 255) / 256)), S), dim3(256), 0, st, src,
                     off, n, raw, cap);
  return hipGetLastError();
}

hipError_t sr_alloc(SrBuffers& b, int S, int cap, int R) {
  DevAlloc A;
  b.S = S; b.cap = cap; b.R = R;
  const size_t n = (size_t)S * cap;
  A(&b.raw, n * sizeof(float4));
  A(&b.raw_n, S * sizeof(int));
  A(&b.tmp_ori, n * sizeof(float));
  A(&b.tmp_sid, n);
  A(&b.tilecnt, (size_t)S * b.ntiles() * R * sizeof(int));
  A(&b.tileF, (size_t)S * b.ntiles() * sizeof(int));
  A(&b.ring_sync, sizeof(int));
  A(&b.sweep_ori, (size_t)S * 2 * sizeof(float));
  A(&b.full, n * sizeof(float4));
  A(&b.n_full, S * sizeof(int));
  A(&b.curv, n * sizeof(float));
  A(&b.picked, n);
  A(&b.sortind, n * sizeof(int));
  A(&b.label, n);
  A(&b.ring_se, (size_t)S * 2 * R * sizeof(int));
  A(&b.st_sharp, (size_t)S * R * kSharpPerRing * sizeof(int));
  A(&b.st_lsharp, (size_t)S * R * kLessSharpPerRing * sizeof(int));
  A(&b.st_flat, (size_t)S * R * kFlatPerRing * sizeof(int));
  A(&b.st_lflat, (size_t)S * R * kRingCap * sizeof(float4));
  A(&b.st_cnt, (size_t)S * R * 4 * sizeof(int));
  A(&b.st_cand, (size_t)S * R * kRingCap * sizeof(uint16_t));
  A(&b.st_ncand, (size_t)S * R * sizeof(int));
  A(&b.sharp, (size_t)S * R * kSharpPerRing * sizeof(float4));
  A(&b.lsharp, (size_t)S * R * kLessSharpPerRing * sizeof(float4));
  A(&b.flat, (size_t)S * R * kFlatPerRing * sizeof(float4));
  A(&b.lflat, n * sizeof(float4));
  A(&b.cnt, (size_t)S * 4 * sizeof(int));
  A(&b.err, S * sizeof(int));
  A(&b.sel_big, S * sizeof(int));
  A(&b.sel_list, (2 + 2 * (size_t)S) * sizeof(int));
  A(&b.st_loff, (size_t)S * R * sizeof(int));
  b.big_stride = next_pow2(cap);
  A(&b.big_keys, (size_t)kBigSlots * b.big_stride * sizeof(uint64_t));
  A(&b.big_sidx, (size_t)kBigSlots * b.big_stride * sizeof(int));
  A(&b.big_cand, (size_t)kBigSlots * b.big_stride * sizeof(int));
  if (A.err != hipSuccess) sr_free(b);
  return A.err;
}

void sr_free(SrBuffers& b) {
  void* ptrs[] = {b.raw, b.raw_n, b.tmp_ori, b.tmp_sid, b.tilecnt, b.tileF, b.ring_sync, b.sweep_ori, b.full, b.n_full, b.curv,
                  b.picked, b.sortind, b.label, b.ring_se, b.st_sharp, b.st_lsharp, b.st_flat,
                  b.st_lflat, b.st_cnt, b.st_cand, b.st_ncand, b.sharp, b.lsharp, b.flat, b.lflat, b.cnt, b.err, b.sel_big, b.sel_list, b.st_loff, b.big_keys, b.big_sidx, b.big_cand};
  for (void* q : ptrs)
    if (q) HIPCHK(hipFree(q));
  b = SrBuffers();
}

// k_sr_ring_fused's tiles wait for the other tiles of their sweep, so a launch is safe only when a
// whole sweep's tiles can be resident at once: its workgroups per CU (the occupancy its registers
// and LDS allow, queried once per device) times the CUs.  Other streams' kernels may hold slots
// for a while, but they never wait on this launch, so the bound is the idle device's.
int sr_ring_fused_capacity() {
  static int cap[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sr_ring_fused, kSrThreads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      per_cu = cus = 0;
    cap[dev] = std::max(1, per_cu * cus);  // (1: a failed query keeps the two-kernel form below)
  }
  return cap[dev];
}

void sr_launch(const SrBuffers& b, const SrParams& p, hipStream_t st, Prof* prof, hipEvent_t sorted) {
  auto mark = [&](const char* n) { if (prof) prof->mark(n); };
  if (p.imu) {  // (the tile-parallel ring sorts clear them in their tile 0)
    HIPCHK(hipMemsetAsync(b.ring_se, 0, (size_t)b.S * 2 * b.R * sizeof(int), st));
    HIPCHK(hipMemsetAsync(b.err, 0, (size_t)b.S * sizeof(int), st));
  }
  mark("sr_memset");
  if (p.imu) {
    hipLaunchKernelGGL(k_sr_ring_sort<true>, dim3(b.S), dim3(kSrThreads), 0, st, b, p);
  } else {
    const int rtiles = (b.cap + kRingTile - 1) / kRingTile;  // <= b.ntiles(): tilecnt rows fit
    // (a margin of 2: a sweep's tiles fit in half the co-resident slots; HDL-64E's 160k-point
    // sweeps are 79 tiles against several per CU x 256 CUs on MI355X)
    if (kSrRingFused && b.S >= kSrRingFusedMin && 2 * rtiles <= sr_ring_fused_capacity()) {
      HIPCHK(hipMemsetAsync(b.ring_sync, 0, sizeof(int), st));
      HIPCHK(hipMemsetAsync(b.tilecnt, 0xff, (size_t)b.S * rtiles * b.R * sizeof(int), st));
      HIPCHK(hipMemsetAsync(b.tileF, 0xff, (size_t)b.S * rtiles * sizeof(int), st));
      hipLaunchKernelGGL(k_sr_ring_fused, dim3(rtiles * b.S), dim3(kSrThreads), 0, st, b, p, rtiles);
    } else {
      hipLaunchKernelGGL(k_sr_ring_count, dim3(rtiles, b.S), dim3(kSrThreads), 0, st, b, p);
      hipLaunchKernelGGL(k_sr_ring_scatter, dim3(rtiles, b.S), dim3(kSrThreads), 0, st, b, p);
    }
  }
  mark("k_sr_ring_sort");
  if (sorted) HIPCHK(hipEventRecord(sorted, st));  // the ring-sorted full cloud is final here
  hipLaunchKernelGGL(k_sr_features, dim3((b.cap + kFeatSpan - 1) / kFeatSpan, b.S), dim3(kFeatTile), 0,
                     st, b, p);
  mark("k_sr_features");
  hipLaunchKernelGGL(k_sr_pick, dim3((b.R + kPickWaves - 1) / kPickWaves, b.S), dim3(64 * kPickWaves), 0, st, b, p);
  hipLaunchKernelGGL(k_sr_ringvg, dim3(b.R, b.S), dim3(kSelThreads), LOAM_RINGVG_PAD, st, b, p);
  // (the sweeps k_sr_pick routed on, from its list: a sweep with an empty ring or a ring beyond
  // kPickCap points; a small grid when there are none)
  hipLaunchKernelGGL((k_sr_select<kRingCap, 1>), dim3(b.R, std::min(b.S, kSelListGrid)), dim3(kSelThreads), 0, st, b, p);
  hipLaunchKernelGGL((k_sr_select<16, 2>), dim3(kBigSlots), dim3(kSelThreads), 0, st, b, p);
  mark("k_sr_select");
  hipLaunchKernelGGL(k_sr_compact, dim3(b.R, b.S), dim3(256), 0, st, b, p);
  mark("k_sr_compact");
}

}  // namespace loam

