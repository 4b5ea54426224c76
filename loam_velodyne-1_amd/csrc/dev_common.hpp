// Device-side building blocks shared by the SR / OD / MP kernels (gfx950, wave64).
//
// Numerics: every kernel is compiled with -ffp-contract=off so that float expressions round
// exactly like the reference build (x86-64 SSE, no FMA).  The reference's unqualified libm calls
// bind the C double functions (ROS Indigo toolchain, see oracle/oracle.cpp header), so the helpers
// below evaluate trig in double and callers round once on assignment to float, mirroring
// src/laserOdometry.cpp / src/laserMapping.cpp; scanRegistration's `using std::atan2` calls are
// float (src/scanRegistration.cpp:51-53).
#ifndef LOAM_DEV_COMMON_HPP
#define LOAM_DEV_COMMON_HPP

#include <hip/hip_runtime.h>
#include <stdint.h>

#define LOAM_HD __host__ __device__ __forceinline__
#define LOAM_D __device__ __forceinline__

// Index bounds checks of the batch-scaled buffers (the per-problem strides of the association,
// coefficient and 5-NN stores): compiled in only by `make checked` (libloam_hip_checked.so, run
// through LOAM_HIP_LIB), where a violated bound prints one line and the kernel carries on.
#ifdef LOAM_BOUNDS_CHECK
#define LOAM_CHECK(cond, a, b)                                                                      \
  do {                                                                                              \
    if (!(cond)) printf("LOAM_CHECK %s:%d %s (%lld, %lld)\n", __FILE__, __LINE__, #cond, (long long)(a), \
                        (long long)(b));                                                            \
  } while (0)
#else
#define LOAM_CHECK(cond, a, b) ((void)0)
#endif

// Phase stamps of the last-workgroup kernels (k_od_rows_small, k_mp_lm_small): compiled in only by
// the diagnostic build (tools/build_variant.sh NAME -DLOAM_PHASES, read by tools/phase_stream.py);
// the product build has none.  Clock: s_memrealtime (100 MHz, one counter for the whole chip, so
// stamps of different workgroups compare).  Per launch: sum[k][0] rows = last arrival - first
// workgroup start, [1] hand-off (arrival -> after the acquire), [2] fixed-order partial sum, [3] the
// step (6x6 solve, eigen at iteration 0), [4] sum over workgroups of (arrival - own start), [5]
// workgroups, [6] launches; k_mp_lm_small also [7] / [8] the sum over its query waves of the 5-NN
// search / the fit + row time, [9] those waves, [10] the last workgroup start - s0, [11] the longest
// query wave; k = 0 for the first L-M iteration, 1 for the others.
struct PhaseAcc {
  unsigned long long s0, s1, s2;  // per launch: first start, last start, longest query wave
  unsigned long long sum[2][12];
};
#ifdef LOAM_PHASES
#define LOAM_PH(...) __VA_ARGS__
#else
#define LOAM_PH(...)
#endif

namespace loamdev {

constexpr int kWave = 64;

LOAM_HD double D(float x) { return (double)x; }
// two consecutive ints (4-byte aligned) as one 8-byte load: one address per lane for the gather
// unit instead of two (hash bucket ranges start[h], start[h + 1])
struct __attribute__((aligned(4))) IntPair4 { int x, y; };
LOAM_D int2 load_pair(const int* p) {
  const IntPair4 v = *reinterpret_cast<const IntPair4*>(p);
  return make_int2(v.x, v.y);
}
// PCL 1.7.1 VoxelGrid's "leaf size too small" test (output = input when the (int64) voxel count
// dx·dy·dz of the bbox exceeds INT_MAX), written without PCL's undefined cases: PCL multiplies
// three int64 extents (overflows for spans beyond ~4·10^5 km at 0.2 m) and converts the scaled
// bbox corners to int; both count as "too small" here.  Identical to PCL wherever PCL is defined.
// The oracle restates it (oracle_math.hpp vg_leaf_too_small).
LOAM_HD bool vg_leaf_too_small(const float* mn, const float* mx, float inv) {
  int64_t e[3];
  for (int d = 0; d < 3; ++d) {
    const float sp = (mx[d] - mn[d]) * inv, lo = mn[d] * inv, hi = mx[d] * inv;
    if (!(sp < 2147483648.0f) || !(lo >= -2147483648.0f) || !(hi < 2147483648.0f)) return true;
    e[d] = (int64_t)sp + 1;
  }
  const int64_t xy = e[0] * e[1];  // each factor <= 2^31: no overflow
  return xy > (int64_t)0x7fffffff || xy * e[2] > (int64_t)0x7fffffff;
}
// Per-workgroup partials handed to the last workgroup to finish (k_od_rows_small, k_mp_lm_small,
// k_mp_iter_wide), in the form MI355X_MICROARCH.md lists as valid without a per-workgroup release:
// each partial stored write-through (agent-scope relaxed = sc1) and drained by its wave before the
// workgroup barrier, then ONE lane's relaxed agent-scope add on the done counter; the last
// workgroup (told by the add's return value) acquires at agent scope once and reads the partials
// with sc1 loads.  A __threadfence() per workgroup (L2 write-back + invalidate) cost several us each.
// The hand-off relies on gfx9's vmcnt counting stores as well as loads (gfx10+ counts stores in a
// separate vscnt, where this drain would not wait for them): CDNA3 / CDNA4 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "store_partial's write-through hand-off is written for gfx942 / gfx950 (vmcnt covers stores)"
#endif
LOAM_D void store_partial(double* dst, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
#ifdef LOAM_PHASES
LOAM_D unsigned long long ph_now() { return __builtin_amdgcn_s_memrealtime(); }
// every workgroup at its start (one lane)
LOAM_D void ph_start(PhaseAcc* a, unsigned long long t0) {
  atomicMin(&a->s0, t0);
  atomicMax(&a->s1, t0);
}
// every workgroup at its arrival (one lane)
LOAM_D void ph_arrive(PhaseAcc* a, int k, unsigned long long t0, unsigned long long t1) {
  atomicAdd(&a->sum[k][4], t1 - t0);
  atomicAdd(&a->sum[k][5], 1ull);
}
// a query wave's search / fit times (one lane)
LOAM_D void ph_query(PhaseAcc* a, int k, unsigned long long tnn, unsigned long long tfit) {
  atomicAdd(&a->sum[k][7], tnn);
  atomicAdd(&a->sum[k][8], tfit);
  atomicAdd(&a->sum[k][9], 1ull);
  atomicMax(&a->s2, tnn + tfit);
}
// the last workgroup once its step is done (one lane): the launch's phases, then s0 reset
LOAM_D void ph_last(PhaseAcc* a, int k, unsigned long long t1, unsigned long long t2, unsigned long long t3,
                    unsigned long long t4) {
  const unsigned long long s0 = __hip_atomic_load(&a->s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long s1 = __hip_atomic_load(&a->s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long s2 = __hip_atomic_load(&a->s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  atomicAdd(&a->sum[k][10], s1 - s0);
  atomicAdd(&a->sum[k][11], s2);
  __hip_atomic_store(&a->s1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&a->s2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  atomicAdd(&a->sum[k][0], t1 - s0);
  atomicAdd(&a->sum[k][1], t2 - t1);
  atomicAdd(&a->sum[k][2], t3 - t2);
  atomicAdd(&a->sum[k][3], t4 - t3);
  atomicAdd(&a->sum[k][6], 1ull);
  __hip_atomic_store(&a->s0, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#endif
LOAM_D bool arrive_last(int* done, int G) {  // one lane; true for the last of G arrivals
  return __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
}
LOAM_HD double dsin(float x) { return sin((double)x); }
LOAM_HD double dcos(float x) { return cos((double)x); }
// sin and cos of one float argument in double; on the device one ocml sincos (the same argument
// reduction and polynomials as its sin and cos, so the same values, for half the work)
LOAM_HD void dsincos(float x, double& s, double& c) {
#ifdef __HIP_DEVICE_COMPILE__
  sincos((double)x, &s, &c);
#else
  s = sin((double)x);
  c = cos((double)x);
#endif
}
LOAM_HD double rad2deg(double r) { return r * 180.0 / M_PI; }

// squared distance in the reference's float order (dx*dx + dy*dy) + dz*dz
LOAM_HD float sqdist(float ax, float ay, float az, float bx, float by, float bz) {
  float dx = ax - bx, dy = ay - by, dz = az - bz;
  return dx * dx + dy * dy + dz * dz;
}

// ------------------------------------------------------------------ wave primitives
LOAM_D int lane_id() { return __lane_id(); }
LOAM_D uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Workgroup coordinates of a 2-D (chunk, problem) grid renumbered so that the chunks of one
// problem run on one XCD.  The dispatcher deals workgroups round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, "Workgroup dispatch"), so linear id L lands on XCD L % 8; logical id
// = (XCD-major rank of L) keeps a problem's consecutive chunks in one XCD's 4 MiB L2, where its
// clouds / hash are shared, instead of fetching them into all eight.  A bijection on the grid:
// placement only, never correctness.
struct XcdBlock { int x, y; };
LOAM_D XcdBlock xcd_block() {
  const int gx = gridDim.x, total = gx * gridDim.y;
  const int L = blockIdx.x + blockIdx.y * gx;
  const int x8 = L & 7, i = L >> 3, q = total >> 3, r = total & 7;
  const int logical = x8 < r ? x8 * (q + 1) + i : r * (q + 1) + (x8 - r) * q + i;
  return {logical % gx, logical / gx};
}

template <typename T>
LOAM_D T wave_sum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
LOAM_D int wave_min_i(int v) {
  for (int o = 32; o > 0; o >>= 1) { int w = __shfl_xor(v, o, 64); v = w < v ? w : v; }
  return v;
}
LOAM_D int wave_max_i(int v) {
  for (int o = 32; o > 0; o >>= 1) { int w = __shfl_xor(v, o, 64); v = w > v ? w : v; }
  return v;
}
LOAM_D uint64_t wave_min_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}
LOAM_D float wave_min_f(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
LOAM_D float wave_max_f(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// inclusive prefix sum across the wave
LOAM_D int wave_incl_scan(int v) {
  for (int o = 1; o < 64; o <<= 1) {
    int w = __shfl_up(v, o, 64);
    if (lane_id() >= o) v += w;
  }
  return v;
}

// ---- cross-lane without the LDS crossbar (gfx950): DPP row operations fused into the VALU op,
// and v_permlane16_swap / v_permlane32_swap for the 16- and 32-lane exchanges.  __shfl_xor /
// __shfl_up compile to ds_bpermute_b32: an address VGPR, an LDS round trip and a wait per step
// (214 of them in the association kernel).  The _x forms below take an identity `old` for the
// lanes a DPP read cannot reach; they are meant for call sites where the whole wave (or, for the
// half forms, the whole 32-lane half) is active.  Only order-free operations (min, max, integer
// sums / scans) are offered, so results are bit-identical to the shuffle forms.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E;         // quad_perm [1,0,3,2] / [2,3,0,1]
constexpr int kDppHalfMirror = 0x141, kDppRor8 = 0x128; // row_half_mirror (8 lanes), row_ror:8 (= xor 8)
constexpr int kDppShr1 = 0x111, kDppShr2 = 0x112, kDppShr3 = 0x113, kDppShr4 = 0x114, kDppShr8 = 0x118;
constexpr int kDppBcast15 = 0x142, kDppBcast31 = 0x143;
template <int CTRL, int ROW = 0xf, int BANK = 0xf>
LOAM_D uint32_t dpp_u32(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW, BANK, false);
}
// v and its partner lane l ^ 16 (first) / l ^ 32 (second) in one swap: min / max take both
LOAM_D uint32_t min_x16(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return r[0] < r[1] ? r[0] : r[1];
}
LOAM_D uint32_t min_x32(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return r[0] < r[1] ? r[0] : r[1];
}
// the value of lane (l ^ m) for a wave-uniform m in {1, 2, 4, 8, 16, 32} (others: __shfl_xor),
// bit-identical to __shfl_xor(v, m, 64) with the whole wave active
LOAM_D uint32_t xor_u32(uint32_t v, int m) {
  switch (m) {
    case 1: return dpp_u32<kDppXor1>(v, v);
    case 2: return dpp_u32<kDppXor2>(v, v);
    case 4: {  // banks 0 / 2 of each row read lane + 4 (row_shl:4), banks 1 / 3 lane - 4 (row_shr:4)
      const uint32_t t = dpp_u32<0x104, 0xf, 0x5>(v, v);
      return dpp_u32<kDppShr4, 0xf, 0xa>(t, v);
    }
    case 8: return dpp_u32<kDppRor8>(v, v);
    case 16: {
      const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
      return (__lane_id() & 16) ? r[0] : r[1];
    }
    case 32: {
      const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
      return (__lane_id() & 32) ? r[0] : r[1];
    }
    default: return (uint32_t)__shfl_xor((int)v, m, 64);
  }
}
LOAM_D double xor_f64(double v, int m) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint64_t r = ((uint64_t)xor_u32((uint32_t)(u >> 32), m) << 32) | xor_u32((uint32_t)u, m);
  return __builtin_bit_cast(double, r);
}
// min over the 32-lane half (HALF) or the wave
template <bool HALF = false>
LOAM_D uint32_t wave_min_u32_x(uint32_t v) {
  v = min(v, dpp_u32<kDppXor1>(~0u, v));
  v = min(v, dpp_u32<kDppXor2>(~0u, v));
  v = min(v, dpp_u32<kDppHalfMirror>(~0u, v));
  v = min(v, dpp_u32<kDppRor8>(~0u, v));
  v = min_x16(v);
  if constexpr (!HALF) v = min_x32(v);
  return v;
}
// 64-bit keys: the high words' minimum, then the low words' among the lanes holding it
template <bool HALF = false>
LOAM_D uint64_t wave_min_u64_x(uint64_t v) {
  const uint32_t hi = wave_min_u32_x<HALF>((uint32_t)(v >> 32));
  const uint32_t lo = wave_min_u32_x<HALF>((uint32_t)(v >> 32) == hi ? (uint32_t)v : ~0u);
  return ((uint64_t)hi << 32) | lo;
}
// float minimum (fminf semantics on non-NaN values: -0 and +0 compare equal either way)
template <bool HALF = false>
LOAM_D float wave_min_f_x(float v) {
  constexpr uint32_t kInf = 0x7f800000u;
  v = fminf(v, __uint_as_float(dpp_u32<kDppXor1>(kInf, __float_as_uint(v))));
  v = fminf(v, __uint_as_float(dpp_u32<kDppXor2>(kInf, __float_as_uint(v))));
  v = fminf(v, __uint_as_float(dpp_u32<kDppHalfMirror>(kInf, __float_as_uint(v))));
  v = fminf(v, __uint_as_float(dpp_u32<kDppRor8>(kInf, __float_as_uint(v))));
  {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  if constexpr (!HALF) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  return v;
}
// float maximum, likewise
LOAM_D float wave_max_f_x(float v) {
  constexpr uint32_t kNInf = 0xff800000u;
  v = fmaxf(v, __uint_as_float(dpp_u32<kDppXor1>(kNInf, __float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(dpp_u32<kDppXor2>(kNInf, __float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(dpp_u32<kDppHalfMirror>(kNInf, __float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(dpp_u32<kDppRor8>(kNInf, __float_as_uint(v))));
  {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  return v;
}
// the workgroup's maximum of an unsigned value (DPP wave maxima, one LDS exchange); every thread
// of the workgroup must call it
template <int NT>
LOAM_D uint32_t block_max_u32(uint32_t v) {
  constexpr int NW = NT / 64;
  __shared__ uint32_t bm[NW];
  const uint32_t m = ~wave_min_u32_x(~v);
  if (lane_id() == 0) bm[threadIdx.x >> 6] = m;
  __syncthreads();
  uint32_t r = bm[0];
  for (int i = 1; i < NW; ++i) r = bm[i] > r ? bm[i] : r;
  __syncthreads();
  return r;
}
// the workgroup's bounding box: the six minima / maxima reduced together (two barriers instead of
// two per value); every thread of the workgroup must call it, and gets the box
template <int NT>
LOAM_D void block_bbox(float (&mn)[3], float (&mx)[3]) {
  constexpr int NW = NT / 64;
  __shared__ float bb[6][NW];
  const int w = threadIdx.x >> 6, l = lane_id();
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float a = wave_min_f_x(mn[d]), b = wave_max_f_x(mx[d]);
    if (l == 0) { bb[d][w] = a; bb[3 + d][w] = b; }
  }
  __syncthreads();
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float a = bb[d][0], b = bb[3 + d][0];
    for (int v = 1; v < NW; ++v) { a = fminf(a, bb[d][v]); b = fmaxf(b, bb[3 + d][v]); }
    mn[d] = a;
    mx[d] = b;
  }
  __syncthreads();
}
// inclusive prefix sum over the wave (HALF: over each 32-lane half), the row-shift / row-broadcast
// ladder: lanes beyond a row's start read 0
template <bool HALF = false>
LOAM_D int wave_incl_scan_x(int v) {
  const uint32_t u = (uint32_t)v;
  uint32_t s = u + dpp_u32<kDppShr1>(0u, u);
  s += dpp_u32<kDppShr2>(0u, u);
  s += dpp_u32<kDppShr3>(0u, u);
  s += dpp_u32<kDppShr4, 0xf, 0xe>(0u, s);   // lanes 4..15 of each row
  s += dpp_u32<kDppShr8, 0xf, 0xc>(0u, s);   // lanes 8..15
  s += dpp_u32<kDppBcast15, 0xa, 0xf>(0u, s); // rows 1 and 3: + lane 15 of rows 0 / 2
  if constexpr (!HALF) s += dpp_u32<kDppBcast31, 0xc, 0xf>(0u, s);  // rows 2, 3: + lane 31
  return (int)s;
}

LOAM_D int wave_incl_max(int v) {
  for (int o = 1; o < 64; o <<= 1) {
    int w = __shfl_up(v, o, 64);
    if (lane_id() >= o) v = max(v, w);
  }
  return v;
}

// ------------------------------------------------------------------ block primitives
// inclusive max-scan of one int per thread over a block of NT threads (thread order); returns
// the block maximum in `total`.  scratch: at least NT/64 + 1 ints of LDS.
template <int NT>
LOAM_D int block_incl_max(int v, int* scratch, int& total) {
  const int nw = NT / 64, w = threadIdx.x >> 6, l = lane_id();
  int incl = wave_incl_max(v);
  if (l == 63) scratch[w] = incl;
  __syncthreads();
  int before = -0x7fffffff;
  for (int k = 0; k < w; ++k) before = max(before, scratch[k]);
  int tot = -0x7fffffff;
  for (int k = 0; k < nw; ++k) tot = max(tot, scratch[k]);
  total = tot;
  __syncthreads();
  return max(before, incl);
}

// exclusive scan of one int per thread over a block of NT threads; returns the block total.
// scratch: at least NT/64 ints of LDS.
template <int NT>
LOAM_D int block_excl_scan(int v, int* scratch, int& total) {
  const int nw = NT / 64, w = threadIdx.x >> 6, l = lane_id();
  int incl = wave_incl_scan_x(v);
  if (l == 63) scratch[w] = incl;
  __syncthreads();
  if (w == 0) {
    int s = l < nw ? scratch[l] : 0;
    int si = wave_incl_scan_x(s);
    if (l < nw) scratch[l] = si - s;
    if (l == nw - 1) scratch[nw] = si;
  }
  __syncthreads();
  int r = incl - v + scratch[w];
  total = scratch[nw];
  __syncthreads();
  return r;
}

template <int NT, typename T, typename Op>
LOAM_D T block_reduce(T v, T* scratch, Op op) {
  const int nw = NT / 64, w = threadIdx.x >> 6, l = lane_id();
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  if (l == 0) scratch[w] = v;
  __syncthreads();
  T r = scratch[0];
  for (int i = 1; i < nw; ++i) r = op(r, scratch[i]);
  __syncthreads();
  return r;
}

// In-place butterfly reduce-scatter of 28 (padded to 32) per-lane doubles over the wave: after
// the call, a[0] of lanes 2v and 2v+1 holds the wave sum of value v.  Step s exchanges with lane
// ^ (32 >> s) and keeps the half of the remaining values selected by that lane bit.
LOAM_D void wave_reduce_scatter_28(double (&a)[28]) {
  const int lane = lane_id();
  double v[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k] = k < 28 ? a[k] : 0.0;
#pragma unroll
  for (int h = 16; h >= 1; h >>= 1) {  // 32 -> 16 -> ... -> 1 values, partner lane ^ (2h)
    const bool upper = (lane & (2 * h)) != 0;
#pragma unroll
    for (int k = 0; k < h; ++k) {
      const double send = upper ? v[k] : v[h + k];
      const double keep = upper ? v[h + k] : v[k];
      v[k] = keep + xor_f64(send, 2 * h);
    }
  }
  a[0] = v[0] + xor_f64(v[0], 1);
}

// ------------------------------------------------------------------ LDS bitonic sort (ascending)
// sorts n64 = power of two 64-bit keys in LDS with the whole block; pad with ~0ull.
template <int NT>
LOAM_D void block_bitonic_sort(uint64_t* k, int n64) {
  // a stage with stride <= 64 touches, per wave, only the 128-element blocks its pairs span: two
  // consecutive such stages are separated by a wave-level fence instead of a workgroup barrier
  for (int size = 2; size <= n64; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (n64 >> 1); t += NT) {
        int lo = 2 * t - (t & (stride - 1));
        int hi = lo + stride;
        bool up = ((lo & size) == 0);
        uint64_t a = k[lo], b = k[hi];
        if ((a > b) == up) { k[lo] = b; k[hi] = a; }
      }
      const int next = stride > 1 ? stride >> 1 : (size << 1 <= n64 ? size : 0);
      if (stride > 64 || next > 64 || next == 0) {
        __syncthreads();
      } else {
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}

// ------------------------------------------------------------------ register bitonic sort (ascending)
// Sorts the n (power of two) 64-bit keys of k[0, n) in LDS with a block of NT threads: the keys
// move into registers (E = n / NT per thread, element g = tid * E + e), strides < E are compare-
// exchanges inside a thread, strides < 64 E are lane exchanges (shuffles) inside a wave, and only
// strides >= 64 E go through LDS — 3 of the 66 stages of a 2048-key sort, against a workgroup
// barrier per stage for the plain LDS network.  k is the LDS scratch of those stages and receives
// the sorted keys.  The initial placement of a key is irrelevant (a sort is a permutation), so the
// loads are coalesced.
// (the register sorts' runtime strides: ds_bpermute; xor_u32's switch per exchange measured slower
// there, k_sr_select 1.55 -> 2.53 ms/step at batch 1024)
// (DPP / permlane stages here measured slower than ds_bpermute: k_sr_select 1.54 -> 1.65 ms/step at
// batch 1024 with a switch per stage in the wave sorts, 2.53 with one per exchange)
LOAM_D uint64_t shfl_xor_u64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
template <int E, int S>
LOAM_D void reg_cmpx_intra(uint64_t (&v)[E], int base, int size) {
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if constexpr (S < E) {
      if ((e & S) == 0) {
        const bool up = ((base + e) & size) == 0;
        const uint64_t a = v[e], b = v[e + S];
        const bool sw = (a > b) == up;
        v[e] = sw ? b : a;
        v[e + S] = sw ? a : b;
      }
    }
  }
}
// WAVE: one wave sorts alone (NT = 64; every stride stays inside the wave, no workgroup barrier)
template <int NT, int E, bool WAVE = false>
LOAM_D void reg_bitonic_sort_n(uint64_t* k, int n) {
  static_assert(!WAVE || NT == 64, "a wave sort has 64 lanes");
  const int lane = __lane_id(), tid = WAVE ? lane : (int)threadIdx.x, base = tid * E;
  constexpr int N = NT * E;
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int g = e * NT + tid;
    v[e] = g < n ? k[g] : ~0ull;
  }
  if (!WAVE) __syncthreads();  // k becomes scratch
  for (int size = 2; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride < E) {
        if (stride == 1) reg_cmpx_intra<E, 1>(v, base, size);
        else if (stride == 2) reg_cmpx_intra<E, 2>(v, base, size);
        else if (stride == 4) reg_cmpx_intra<E, 4>(v, base, size);
        else reg_cmpx_intra<E, 8>(v, base, size);
      } else if (stride < 64 * E) {
        const int m = stride / E;
        const bool lower = (lane & m) == 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool up = ((base + e) & size) == 0;
          const uint64_t o = shfl_xor_u64(v[e], m);
          const bool keep_min = lower == up;
          v[e] = keep_min ? (o < v[e] ? o : v[e]) : (o > v[e] ? o : v[e]);
        }
      } else {
        const int m = stride / E;
        const bool lower = (tid & m) == 0;
#pragma unroll
        for (int e = 0; e < E; ++e) k[e * NT + tid] = v[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool up = ((base + e) & size) == 0;
          const uint64_t o = k[e * NT + (tid ^ m)];
          const bool keep_min = lower == up;
          v[e] = keep_min ? (o < v[e] ? o : v[e]) : (o > v[e] ? o : v[e]);
        }
        __syncthreads();
      }
    }
  }
  if (WAVE) __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (base + e < n) k[base + e] = v[e];
  if (WAVE) {
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}
// one wave sorts n <= 512 keys of k (ascending); the other waves do not take part
LOAM_D void wave_sort_u64(uint64_t* k, int n) {
  if (n <= 64) reg_bitonic_sort_n<64, 1, true>(k, n);
  else if (n <= 128) reg_bitonic_sort_n<64, 2, true>(k, n);
  else if (n <= 256) reg_bitonic_sort_n<64, 4, true>(k, n);
  else reg_bitonic_sort_n<64, 8, true>(k, n);
}
// n: power of two <= NT * EMAX (EMAX a power of two <= 16)
template <int NT, int EMAX>
LOAM_D void reg_bitonic_sort(uint64_t* k, int n) {
  if (n <= NT || EMAX == 1) reg_bitonic_sort_n<NT, 1>(k, n);
  else if (n <= 2 * NT || EMAX == 2) reg_bitonic_sort_n<NT, (EMAX < 2 ? EMAX : 2)>(k, n);
  else if (n <= 4 * NT || EMAX == 4) reg_bitonic_sort_n<NT, (EMAX < 4 ? EMAX : 4)>(k, n);
  else if (n <= 8 * NT || EMAX == 8) reg_bitonic_sort_n<NT, (EMAX < 8 ? EMAX : 8)>(k, n);
  else reg_bitonic_sort_n<NT, (EMAX < 16 ? EMAX : 16)>(k, n);
}

// ------------------------------------------------------------------ block radix sort (stable)
// LSD radix sort of n <= NT*E (key, value) pairs held in LDS, 4-bit digits, over the low `nbits`
// bits of the keys (the caller passes the bits its keys can differ in).  Blocked arrangement:
// thread t ranks items [t*E, t*E+E) — digit counters packed in two 64-bit registers (8-bit fields),
// one packed (16-bit pair) wave scan + one cross-wave scan per pass, scatter to the other buffer.
// Stable, so equal keys keep their input order.  Returns 0 when the result is in (ka, va), 1 when
// in (kb, vb).  sc: LDS scratch of (NT/64 + 1) * 8 words.  E <= 255, n < 65536.
template <int NT, int E>
LOAM_D int block_radix_sort_kv(uint32_t* ka, uint16_t* va, uint32_t* kb, uint16_t* vb, int n, int nbits,
                               uint32_t* sc) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
  int cur = 0;
  for (int shift = 0; shift < nbits; shift += 4) {
    const uint32_t* ks = cur ? kb : ka;
    const uint16_t* vs = cur ? vb : va;
    uint32_t* kd = cur ? ka : kb;
    uint16_t* vd = cur ? va : vb;
    uint32_t k[E];
    uint32_t meta[E];  // value | rank in thread << 16 | digit << 24 | valid << 28
    uint64_t clo = 0, chi = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int g = tid * E + e;
      k[e] = 0;
      meta[e] = 0;
      if (g < n) {
        k[e] = ks[g];
        const uint32_t d = (k[e] >> shift) & 15u;
        const int sh = (int)(d & 7u) * 8;
        const uint64_t c = d < 8 ? clo : chi;
        meta[e] = (uint32_t)vs[g] | ((uint32_t)((c >> sh) & 255u) << 16) | (d << 24) | (1u << 28);
        const uint64_t c2 = c + (1ull << sh);
        if (d < 8) clo = c2; else chi = c2;
      }
    }
    uint32_t p[8], inc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // counts of digits 2i, 2i+1 as 16-bit pairs
      const uint64_t c = i < 4 ? clo : chi;
      const int sh = (2 * i % 8) * 8;
      p[i] = (uint32_t)((c >> sh) & 255u) | ((uint32_t)((c >> (sh + 8)) & 255u) << 16);
      inc[i] = p[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) inc[i] = (uint32_t)wave_incl_scan_x((int)inc[i]);  // (DPP: integer sums, any order)
    if (lane == 63)
#pragma unroll
      for (int i = 0; i < 8; ++i) sc[w * 8 + i] = inc[i];
    __syncthreads();
    if (tid < 8) {
      uint32_t run = 0;
      for (int ww = 0; ww < NW; ++ww) {
        const uint32_t t = sc[ww * 8 + tid];
        sc[ww * 8 + tid] = run;
        run += t;
      }
      sc[NW * 8 + tid] = run;
    }
    __syncthreads();
    // digit bases (exclusive prefix of the 16 totals), folded into the thread's packed prefixes
    uint32_t base = 0;
    uint64_t q[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t tot = sc[NW * 8 + i];
      const uint32_t b0 = base, b1 = base + (tot & 0xffffu);
      base = b1 + (tot >> 16);
      const uint32_t ex = inc[i] - p[i] + sc[w * 8 + i] + (b0 | (b1 << 16));
      if (i % 2 == 0) q[i / 2] = ex; else q[i / 2] |= (uint64_t)ex << 32;
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (meta[e] >> 28) {
        const int d = (int)((meta[e] >> 24) & 15u), wd = d >> 2;
        const uint64_t qq = wd == 0 ? q[0] : (wd == 1 ? q[1] : (wd == 2 ? q[2] : q[3]));
        const int pos = (int)((qq >> ((d & 3) * 16)) & 0xffffu) + (int)((meta[e] >> 16) & 255u);
        kd[pos] = k[e];
        vd[pos] = (uint16_t)(meta[e] & 0xffffu);
      }
    __syncthreads();
    cur ^= 1;
  }
  return cur;
}

// One tile of a stable LSD radix pass through global memory (k_vg_big): thread t holds the tile's
// items [t*E, t*E + E) (valid below n_tile) in k[].  For each valid item, rank[e] = its rank among
// the tile's items with the same digit (key >> shift) & 15, in tile order (blocked = input order,
// so the pass is stable); tot[d] (LDS, 16 words) = the tile's count of digit d.  The same packed
// counters as block_radix_sort_kv.  sc: LDS scratch of (NT/64 + 1) * 8 words; n_tile < 65536.
template <int NT, int E>
LOAM_D void tile_rank4(const uint32_t* k, int shift, int n_tile, uint32_t* sc, uint32_t* tot, int* rank) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
  uint32_t meta[E];  // rank in thread | digit << 8 | valid << 12
  uint64_t clo = 0, chi = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    meta[e] = 0;
    if (tid * E + e < n_tile) {
      const uint32_t d = (k[e] >> shift) & 15u;
      const int sh = (int)(d & 7u) * 8;
      const uint64_t c = d < 8 ? clo : chi;
      meta[e] = (uint32_t)((c >> sh) & 255u) | (d << 8) | (1u << 12);
      const uint64_t c2 = c + (1ull << sh);
      if (d < 8) clo = c2; else chi = c2;
    }
  }
  uint32_t p[8], inc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // counts of digits 2i, 2i+1 as 16-bit pairs
    const uint64_t c = i < 4 ? clo : chi;
    const int sh = (2 * i % 8) * 8;
    p[i] = (uint32_t)((c >> sh) & 255u) | ((uint32_t)((c >> (sh + 8)) & 255u) << 16);
    inc[i] = p[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) inc[i] = (uint32_t)wave_incl_scan_x((int)inc[i]);  // (DPP: integer sums, any order)
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[w * 8 + i] = inc[i];
  __syncthreads();
  if (tid < 8) {
    uint32_t run = 0;
    for (int ww = 0; ww < NW; ++ww) {
      const uint32_t t = sc[ww * 8 + tid];
      sc[ww * 8 + tid] = run;
      run += t;
    }
    tot[2 * tid] = run & 0xffffu;
    tot[2 * tid + 1] = run >> 16;
  }
  __syncthreads();
  uint32_t ex[8];  // packed exclusive prefixes of digits 2i, 2i+1 before this thread
#pragma unroll
  for (int i = 0; i < 8; ++i) ex[i] = inc[i] - p[i] + sc[w * 8 + i];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    rank[e] = -1;
    if (meta[e] >> 12) {
      const int d = (int)((meta[e] >> 8) & 15u);
      uint32_t x = ex[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) x = (d >> 1) == i ? ex[i] : x;
      rank[e] = (int)((x >> ((d & 1) * 16)) & 0xffffu) + (int)(meta[e] & 255u);
    }
  }
  __syncthreads();  // sc is reused by the next call
}

LOAM_HD int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// order-preserving float -> uint32 for non-negative floats (curvature, squared distances)
LOAM_HD uint32_t fkey(float f) { return __builtin_bit_cast(uint32_t, f); }
LOAM_HD int32_t f2i(float f) { return __builtin_bit_cast(int32_t, f); }

// ------------------------------------------------------------------ spatial hash
// Cells are grouped in 4x4x4 blocks: the block is hashed, the cell's position in it is the low 6
// bits.  Three consecutive cells along an axis differ mod 4, so the 27 cells around any cell fall
// in 27 different buckets of any table of >= 64 buckets (no point is listed twice by a 3x3x3
// search), and a neighbourhood's bucket ranges lie in a few 64-entry runs of the table.
LOAM_HD uint32_t cell_hash(int ix, int iy, int iz) {
  uint32_t h = (uint32_t)(ix >> 2) * 73856093u ^ (uint32_t)(iy >> 2) * 19349663u ^ (uint32_t)(iz >> 2) * 83492791u;
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  return (h << 6) | (uint32_t)(ix & 3) | ((uint32_t)(iy & 3) << 2) | ((uint32_t)(iz & 3) << 4);
}
LOAM_HD int cell_of(float v, float inv_h) { return (int)floorf(v * inv_h); }


// ------------------------------------------------------------------ glibc-identical sinf / cosf
// scanRegistration's IMU de-skew calls std::sin / std::cos on floats (src/scanRegistration.cpp:51-53,
// :111-179), which glibc (>= 2.28) evaluates in double with a degree-4/3 polynomial after a
// 2/pi range reduction, the FMA build on FMA hardware (ARM optimized-routines sincosf).  This is a
// restatement of that algorithm with the FMAs placed as that build has them; tests/sincosf_check.cpp
// compares it with the host's glibc on every 3rd float of |x| < 120 (0 mismatches).  Arguments
// beyond 120 (never produced by the IMU angles) fall back to the double functions.
struct SinCosTab {
  double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
LOAM_HD const SinCosTab& sincos_tab(int k) {
  static constexpr SinCosTab t[2] = {
      {0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5,
       -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7,
       -0x1.994eb3774cf24p-13},
      {0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5,
       0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7,
       -0x1.994eb3774cf24p-13}};
  return t[k];
}
LOAM_HD uint32_t sc_abstop12(float x) { return (__builtin_bit_cast(uint32_t, x) >> 20) & 0x7ff; }
LOAM_HD float sincosf_poly(double x, double x2, const SinCosTab& p, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2, s1 = fma(x2, p.s3, p.s2), x7 = x3 * x2, s = fma(x3, p.s1, x);
    return (float)fma(x7, s1, s);
  }
  const double x4 = x2 * x2, c2 = fma(x2, p.c4, p.c3), c1 = fma(x2, p.c1, p.c0), x6 = x4 * x2;
  const double c = fma(x4, p.c2, c1);
  return (float)fma(x6, c2, c);
}
LOAM_HD double sincosf_reduce(double x, int& n) {
  const double r = x * sincos_tab(0).hpi_inv;
  n = ((int32_t)r + 0x800000) >> 24;
  return fma(-(double)n, sincos_tab(0).hpi, x);
}
LOAM_HD float sinf_glibc(float y) {
  double x = y;
  if (sc_abstop12(y) < sc_abstop12(0x1.921FB6p-1f)) {
    if (sc_abstop12(y) < sc_abstop12(0x1p-12f)) return y;
    return sincosf_poly(x, x * x, sincos_tab(0), 0);
  }
  if (!(sc_abstop12(y) < sc_abstop12(120.0f))) return (float)sin((double)y);
  int n;
  x = sincosf_reduce(x, n);
  const double s = (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0;
  return sincosf_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n);
}
LOAM_HD float cosf_glibc(float y) {
  double x = y;
  if (sc_abstop12(y) < sc_abstop12(0x1.921FB6p-1f)) {
    if (sc_abstop12(y) < sc_abstop12(0x1p-12f)) return 1.0f;
    return sincosf_poly(x, x * x, sincos_tab(0), 1);
  }
  if (!(sc_abstop12(y) < sc_abstop12(120.0f))) return (float)cos((double)y);
  int n;
  x = sincosf_reduce(x, n);
  const double s = (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0;
  return sincosf_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n ^ 1);
}

// ------------------------------------------------------------------ glibc-identical atan2f
// scanRegistration's float atan2 (`using std::atan2`, src/scanRegistration.cpp:53) resolves to
// glibc's atan2f, the fdlibm single-precision algorithm (sysdeps/ieee754/flt-32/e_atan2f.c,
// s_atanf.c).  Restated here so the device orientation / relTime / intensity are bit-identical
// to the reference toolchain's (ocml's atan2f differs in the last bit for some inputs);
// tests/test_atan2f.py checks it against the host glibc.
LOAM_HD float atanf_fdlibm(float x) {
  const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
  const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
              aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
              aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
              aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  const int32_t hx = f2i(x), ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c800000) {  // |x| >= 2^26
    if (ix > 0x7f800000) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3ee00000) {   // |x| < 0.4375
    if (ix < 0x39800000) return x;
    id = -1;
  } else {
    x = fabsf(x);
    if (ix < 0x3f980000) {
      if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
      else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
    } else {
      if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
      else { id = 3; x = -1.0f / x; }
    }
  }
  const float z = x * x, w = z * z;
  const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -r : r;
}

LOAM_HD float atan2f_fdlibm(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
              pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
  const int32_t hx = f2i(x), ix = hx & 0x7fffffff;
  const int32_t hy = f2i(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return atanf_fdlibm(y);
  int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    if (m < 2) return y;
    return m == 2 ? pi + tiny : -pi - tiny;
  }
  if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0: return 0.0f;
      case 1: return -0.0f;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int k = (iy - ix) >> 23;
  float z;
  if (k > 26) { z = pi_o_2 + 0.5f * pi_lo; m &= 1; }
  else if (k < -26 && hx < 0) z = 0.0f;
  else z = atanf_fdlibm(fabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

}  // namespace loamdev

// ------------------------------------------------------------------ small dense solvers
// Written for the engine from the published algorithms of the calls the reference makes
// (cv::solve DECOMP_QR, cv::eigen Jacobi, cv::Mat::inv LU, float gemm with double accumulation;
// SURVEY.md appendix A2).  Executed by one lane; float arithmetic in the documented order.
namespace loamla {

LOAM_HD float sgn1(float x) { return x >= 0.0f ? 1.0f : -1.0f; }

// Householder least squares, m x n (m >= n <= 6), row-major A (m*n), b (m); A,b destroyed.
// ws: >= 14 floats of scratch (registers for small per-lane solves, LDS for the 6x6 one)
LOAM_HD bool qr_solve(float* A, float* b, int m, int n, float* x, float* ws) {
  float* v = ws;
  float* h = ws + 8;
  const float eps = 1.1920928955078125e-07f * 10;
#pragma unroll
  for (int l = 0; l < n; ++l) {
    const int len = m - l;
    float nrm = 0.0f;
#pragma unroll
    for (int i = 0; i < len; ++i) { v[i] = A[(l + i) * n + l]; nrm += v[i] * v[i]; }
    const float v0 = v[0];
    v[0] = v[0] + sgn1(v[0]) * sqrtf(nrm);
    nrm = sqrtf(nrm + v[0] * v[0] - v0 * v0);
#pragma unroll
    for (int i = 0; i < len; ++i) v[i] /= nrm;
#pragma unroll
    for (int j = l; j < n; ++j) {
      float dot = 0.0f;
#pragma unroll
      for (int i = l; i < m; ++i) dot += v[i - l] * A[i * n + j];
#pragma unroll
      for (int i = l; i < m; ++i) A[i * n + j] -= 2 * v[i - l] * dot;
    }
    h[l] = v[0] * v[0];
#pragma unroll
    for (int i = 1; i < len; ++i) A[(l + i) * n + l] = v[i] / v[0];
  }
#pragma unroll
  for (int l = 0; l < n; ++l) {
    v[0] = 1.0f;
#pragma unroll
    for (int j = 1; j < m - l; ++j) v[j] = A[(j + l) * n + l];
    float dot = 0.0f;
#pragma unroll
    for (int i = l; i < m; ++i) dot += v[i - l] * b[i];
#pragma unroll
    for (int i = l; i < m; ++i) b[i] -= 2 * v[i - l] * dot * h[l];
  }
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
#pragma unroll
    for (int j = n - 1; j > i; --j) b[i] -= b[j] * A[i * n + j];
    if (fabsf(A[i * n + i]) < eps) {
      for (int q = 0; q < n; ++q) x[q] = 0.0f;
      return false;
    }
    b[i] /= A[i * n + i];
  }
  for (int i = 0; i < n; ++i) x[i] = b[i];
  return true;
}

LOAM_HD float hypot_cv(float a, float b) {
  a = fabsf(a);
  b = fabsf(b);
  if (a > b) { b /= a; return a * sqrtf(1 + b * b); }
  if (b > 0) { a /= b; return b * sqrtf(1 + a * a); }
  return 0;
}

template <int N>
LOAM_HD void jacobi_rowmax(const float* A, int* indR, int k) {
  int m = k + 1;
  float mv = fabsf(A[k * N + m]);
  for (int i = k + 2; i < N; ++i) {
    float val = fabsf(A[k * N + i]);
    if (mv < val) { mv = val; m = i; }
  }
  indR[k] = m;
}
template <int N>
LOAM_HD void jacobi_colmax(const float* A, int* indC, int k) {
  int m = 0;
  float mv = fabsf(A[k]);
  for (int i = 1; i < k; ++i) {
    float val = fabsf(A[i * N + k]);
    if (mv < val) { mv = val; m = i; }
  }
  indC[k] = m;
}

// symmetric N x N (A destroyed): W descending, V eigenvectors as rows
template <int N>
LOAM_HD void jacobi(float* A, float* W, float* V, int* iws) {
  int* indR = iws;
  int* indC = iws + N;
  const float eps = 1.1920928955078125e-07f;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) V[i * N + j] = (i == j) ? 1.0f : 0.0f;
  for (int k = 0; k < N; ++k) {
    W[k] = A[k * N + k];
    indR[k] = 0;
    indC[k] = 0;
    if (k < N - 1) jacobi_rowmax<N>(A, indR, k);
    if (k > 0) jacobi_colmax<N>(A, indC, k);
  }
  for (int iters = 0; iters < N * N * 30; ++iters) {
    int k = 0;
    float mv = fabsf(A[indR[0]]);
    for (int i = 1; i < N - 1; ++i) {
      float val = fabsf(A[i * N + indR[i]]);
      if (mv < val) { mv = val; k = i; }
    }
    int l = indR[k];
    for (int i = 1; i < N; ++i) {
      float val = fabsf(A[indC[i] * N + i]);
      if (mv < val) { mv = val; k = indC[i]; l = i; }
    }
    float p = A[k * N + l];
    if (fabsf(p) <= eps) break;
    float y = (float)((W[l] - W[k]) * 0.5);
    float t = fabsf(y) + hypot_cv(p, y);
    float s = hypot_cv(p, t);
    float c = t / s;
    s = p / s;
    t = (p / t) * p;
    if (y < 0) { s = -s; t = -t; }
    A[k * N + l] = 0;
    W[k] -= t;
    W[l] += t;
#define LOAM_ROT(v0, v1)            \
  {                                 \
    float a0 = v0, b0 = v1;         \
    v0 = a0 * c - b0 * s;           \
    v1 = a0 * s + b0 * c;           \
  }
    for (int i = 0; i < k; ++i) LOAM_ROT(A[i * N + k], A[i * N + l]);
    for (int i = k + 1; i < l; ++i) LOAM_ROT(A[k * N + i], A[i * N + l]);
    for (int i = l + 1; i < N; ++i) LOAM_ROT(A[k * N + i], A[l * N + i]);
    for (int i = 0; i < N; ++i) LOAM_ROT(V[k * N + i], V[l * N + i]);
#undef LOAM_ROT
    for (int j = 0; j < 2; ++j) {
      int idx = j == 0 ? k : l;
      if (idx < N - 1) jacobi_rowmax<N>(A, indR, idx);
      if (idx > 0) jacobi_colmax<N>(A, indC, idx);
    }
  }
  for (int k = 0; k < N - 1; ++k) {
    int m = k;
    for (int i = k + 1; i < N; ++i)
      if (W[m] < W[i]) m = i;
    if (k != m) {
      float t = W[m]; W[m] = W[k]; W[k] = t;
      for (int i = 0; i < N; ++i) { float q = V[m * N + i]; V[m * N + i] = V[k * N + i]; V[k * N + i] = q; }
    }
  }
}

// jacobi<3> in registers, bit-identical: only the upper triangle (a01, a02, a12) and the diagonal
// (W) are read by jacobi<N>, and for N = 3 the pivot (k, l) is one of three pairs, so every step is a
// select over the three cases with the same operations in the same order (the row / column maxima
// tracking, the rotation, the final descending sort).  A: row-major 3x3 (symmetric; not modified).
LOAM_HD void jacobi3_reg(const float* A, float* W, float* V) {
  const float eps = 1.1920928955078125e-07f;
  float a01 = A[1], a02 = A[2], a12 = A[5];
  float w0 = A[0], w1 = A[4], w2 = A[8];
  float v00 = 1, v01 = 0, v02 = 0, v10 = 0, v11 = 1, v12 = 0, v20 = 0, v21 = 0, v22 = 1;
  // indR[0] in {1, 2}: the first maximum of |a01|, |a02|; indR[1] = 2; indC[1] = 0; indC[2] in {0, 1}
  int r0 = fabsf(a01) < fabsf(a02) ? 2 : 1, c2 = fabsf(a02) < fabsf(a12) ? 1 : 0;
  for (int iters = 0; iters < 3 * 3 * 30; ++iters) {
    // pivot scan (jacobi<N>: rows k < N - 1 by indR, then columns i >= 1 by indC, strict <)
    int k = 0, l = r0;
    float mv = fabsf(r0 == 1 ? a01 : a02);
    if (mv < fabsf(a12)) { mv = fabsf(a12); k = 1; l = 2; }  // row 1: indR[1] = 2
    if (mv < fabsf(a01)) { mv = fabsf(a01); k = 0; l = 1; }  // column 1: indC[1] = 0
    {
      const float val = fabsf(c2 == 0 ? a02 : a12);           // column 2: indC[2]
      if (mv < val) { mv = val; k = c2; l = 2; }
    }
    const bool p01 = k == 0 && l == 1, p02 = k == 0 && l == 2;  // else (1, 2)
    const float p = p01 ? a01 : (p02 ? a02 : a12);
    if (fabsf(p) <= eps) break;
    const float wk = k == 0 ? w0 : w1, wl = l == 1 ? w1 : w2;
    float y = (float)((wl - wk) * 0.5);
    float t = fabsf(y) + hypot_cv(p, y);
    float s = hypot_cv(p, t);
    const float c = t / s;
    s = p / s;
    t = (p / t) * p;
    if (y < 0) { s = -s; t = -t; }
    // A[k][l] = 0; W[k] -= t; W[l] += t
    if (p01) a01 = 0;
    if (p02) a02 = 0;
    if (!p01 && !p02) a12 = 0;
    if (k == 0) w0 -= t; else w1 -= t;
    if (l == 1) w1 += t; else w2 += t;
    // the one off-diagonal pair the rotation touches: (0, 1) -> (a02, a12) [i > l]; (0, 2) ->
    // (a01, a12) [k < i < l]; (1, 2) -> (a01, a02) [i < k]
    {
      const float x0 = p01 ? a02 : a01, x1 = p02 || p01 ? a12 : a02;
      const float n0 = x0 * c - x1 * s, n1 = x0 * s + x1 * c;
      if (p01) { a02 = n0; a12 = n1; }
      else if (p02) { a01 = n0; a12 = n1; }
      else { a01 = n0; a02 = n1; }
    }
    // eigenvector rows k and l
    {
      const float k0 = k == 0 ? v00 : v10, k1 = k == 0 ? v01 : v11, k2 = k == 0 ? v02 : v12;
      const float l0 = l == 1 ? v10 : v20, l1 = l == 1 ? v11 : v21, l2 = l == 1 ? v12 : v22;
      const float nk0 = k0 * c - l0 * s, nl0 = k0 * s + l0 * c;
      const float nk1 = k1 * c - l1 * s, nl1 = k1 * s + l1 * c;
      const float nk2 = k2 * c - l2 * s, nl2 = k2 * s + l2 * c;
      if (k == 0) { v00 = nk0; v01 = nk1; v02 = nk2; } else { v10 = nk0; v11 = nk1; v12 = nk2; }
      if (l == 1) { v10 = nl0; v11 = nl1; v12 = nl2; } else { v20 = nl0; v21 = nl1; v22 = nl2; }
    }
    // the maxima of rows / columns k and l (jacobi<N> refreshes indR[idx] for idx < N - 1 and
    // indC[idx] for idx > 0; indR[1] and indC[1] are fixed for N = 3)
    if (k == 0) r0 = fabsf(a01) < fabsf(a02) ? 2 : 1;
    if (l == 2) c2 = fabsf(a02) < fabsf(a12) ? 1 : 0;
  }
  // descending selection sort with the eigenvector rows (jacobi<N>'s order)
  auto swap_rows = [](float& wa, float& wb, float& a0, float& a1, float& a2, float& b0, float& b1, float& b2) {
    float q = wa; wa = wb; wb = q;
    q = a0; a0 = b0; b0 = q;
    q = a1; a1 = b1; b1 = q;
    q = a2; a2 = b2; b2 = q;
  };
  {
    int m = 0;
    if (w0 < w1) m = 1;
    if ((m == 0 ? w0 : w1) < w2) m = 2;
    if (m == 1) swap_rows(w0, w1, v00, v01, v02, v10, v11, v12);
    if (m == 2) swap_rows(w0, w2, v00, v01, v02, v20, v21, v22);
  }
  if (w1 < w2) swap_rows(w1, w2, v10, v11, v12, v20, v21, v22);
  W[0] = w0; W[1] = w1; W[2] = w2;
  V[0] = v00; V[1] = v01; V[2] = v02; V[3] = v10; V[4] = v11; V[5] = v12; V[6] = v20; V[7] = v21; V[8] = v22;
}

// jacobi<6> by one whole wave (all 64 lanes active), bit-identical: lane 6r + c (< 36) holds
// A[r][c] and V[r][c] in registers, lanes 0..5 hold W and the tracked row / column maxima (indR,
// indC).  A rotation's element pairs are disjoint, so every affected lane updates at once from its
// partner's value (one cross-lane read each); the pivot scan, the rotation and the tracking scans
// keep the sequential first-maximum order of the one-lane version on wave-uniform values.  The
// one-lane version's chain of dependent LDS accesses per rotation was the iteration-0 cost
// (73-84 us per call).  A (row-major, 36) is read from memory; W, V (rows) are written.
LOAM_D float wl_read(float v, int lane) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane)); }
LOAM_D int wl_readi(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
LOAM_D float wl_perm(float v, int src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src << 2, __builtin_bit_cast(int, v)));
}
LOAM_D void jacobi6_wave(const float* Ain, float* Wout, float* Vout) {
  constexpr int N = 6;
  const float eps = 1.1920928955078125e-07f;
  const int lane = __lane_id();
  const int r = lane / N, c = lane % N;
  float a = lane < N * N ? Ain[lane] : 0.0f;
  float v = lane < N * N ? (r == c ? 1.0f : 0.0f) : 0.0f;
  float w = wl_perm(a, lane < N ? lane * (N + 1) : 0);  // W[k] = A[k][k] on lane k
  // the tracked maxima: row k over A[k][k+1..5] (indR), column k over A[0..k-1][k] (indC)
  auto rowmax = [&](int k) {
    int m = k + 1;
    float mv = fabsf(wl_read(a, k * N + m));
    for (int i = k + 2; i < N; ++i) {
      const float val = fabsf(wl_read(a, k * N + i));
      if (mv < val) { mv = val; m = i; }
    }
    return m;
  };
  auto colmax = [&](int k) {
    int m = 0;
    float mv = fabsf(wl_read(a, k));
    for (int i = 1; i < k; ++i) {
      const float val = fabsf(wl_read(a, i * N + k));
      if (mv < val) { mv = val; m = i; }
    }
    return m;
  };
  int indR[N], indC[N];  // wave-uniform
#pragma unroll
  for (int k = 0; k < N; ++k) {
    indR[k] = k < N - 1 ? rowmax(k) : 0;
    indC[k] = k > 0 ? colmax(k) : 0;
  }
  for (int iters = 0; iters < N * N * 30; ++iters) {
    int k = 0;
    float mv = fabsf(wl_read(a, indR[0]));
    for (int i = 1; i < N - 1; ++i) {
      const float val = fabsf(wl_read(a, i * N + indR[i]));
      if (mv < val) { mv = val; k = i; }
    }
    int l = indR[k];
    for (int i = 1; i < N; ++i) {
      const float val = fabsf(wl_read(a, indC[i] * N + i));
      if (mv < val) { mv = val; k = indC[i]; l = i; }
    }
    k = __builtin_amdgcn_readfirstlane(k);
    l = __builtin_amdgcn_readfirstlane(l);
    const float p = wl_read(a, k * N + l);
    if (fabsf(p) <= eps) break;
    const float Wk = wl_read(w, k), Wl = wl_read(w, l);
    float y = (float)((Wl - Wk) * 0.5);
    float t = fabsf(y) + hypot_cv(p, y);
    float s = hypot_cv(p, t);
    const float cc = t / s;
    s = p / s;
    t = (p / t) * p;
    if (y < 0) { s = -s; t = -t; }
    if (lane == k) w = Wk - t;
    if (lane == l) w = Wl + t;
    // A pairs (v0, v1): (A[i][k], A[i][l]) i < k; (A[k][i], A[i][l]) k < i < l; (A[k][i], A[l][i]) i > l
    int partner = lane, role = 0;  // role 1: v0, 2: v1
    if (c == k && r < k) { role = 1; partner = r * N + l; }
    else if (c == l && r < k) { role = 2; partner = r * N + k; }
    else if (r == k && c > k && c < l) { role = 1; partner = c * N + l; }
    else if (c == l && r > k && r < l) { role = 2; partner = k * N + r; }
    else if (r == k && c > l) { role = 1; partner = l * N + c; }
    else if (r == l && c > l) { role = 2; partner = k * N + c; }
    if (lane >= N * N) role = 0;
    const float other = wl_perm(a, partner);
    if (role == 1) a = a * cc - other * s;
    else if (role == 2) a = other * s + a * cc;
    if (lane == k * N + l) a = 0.0f;
    // V rows k, l
    const int vpart = r == k ? l * N + c : (r == l ? k * N + c : lane);
    const float vo = wl_perm(v, lane < N * N ? vpart : lane);
    if (lane < N * N) {
      if (r == k) v = v * cc - vo * s;
      else if (r == l) v = vo * s + v * cc;
    }
    if (k < N - 1) indR[k] = rowmax(k);
    if (k > 0) indC[k] = colmax(k);
    if (l < N - 1) indR[l] = rowmax(l);
    if (l > 0) indC[l] = colmax(l);
  }
  if (lane < N) Wout[lane] = w;
  if (lane < N * N) Vout[lane] = v;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {  // descending order (rows of V follow)
    for (int k = 0; k < N - 1; ++k) {
      int m = k;
      for (int i = k + 1; i < N; ++i)
        if (Wout[m] < Wout[i]) m = i;
      if (k != m) {
        float tq = Wout[m]; Wout[m] = Wout[k]; Wout[k] = tq;
        for (int i = 0; i < N; ++i) { float q = Vout[m * N + i]; Vout[m * N + i] = Vout[k * N + i]; Vout[k * N + i] = q; }
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// 6 x 6 LU inverse with partial pivoting (A destroyed)
LOAM_HD bool lu_inv6(float* A, float* Inv, float* b) {
  const int n = 6;
  for (int i = 0; i < 36; ++i) b[i] = 0.0f;
  for (int i = 0; i < n; ++i) b[i * n + i] = 1.0f;
  const float eps = 1.1920928955078125e-07f * 10;
  for (int i = 0; i < n; ++i) {
    int k = i;
    for (int j = i + 1; j < n; ++j)
      if (fabsf(A[j * n + i]) > fabsf(A[k * n + i])) k = j;
    if (fabsf(A[k * n + i]) < eps) {
      for (int q = 0; q < 36; ++q) Inv[q] = 0.0f;
      return false;
    }
    if (k != i) {
      for (int j = i; j < n; ++j) { float t = A[i * n + j]; A[i * n + j] = A[k * n + j]; A[k * n + j] = t; }
      for (int j = 0; j < n; ++j) { float t = b[i * n + j]; b[i * n + j] = b[k * n + j]; b[k * n + j] = t; }
    }
    float d = -1 / A[i * n + i];
    for (int j = i + 1; j < n; ++j) {
      float alpha = A[j * n + i] * d;
      for (int q = i + 1; q < n; ++q) A[j * n + q] += alpha * A[i * n + q];
      for (int q = 0; q < n; ++q) b[j * n + q] += alpha * b[i * n + q];
    }
  }
  for (int i = n - 1; i >= 0; --i)
    for (int j = 0; j < n; ++j) {
      float s = b[i * n + j];
      for (int q = i + 1; q < n; ++q) s -= A[i * n + q] * b[q * n + j];
      b[i * n + j] = s / A[i * n + i];
    }
  for (int q = 0; q < 36; ++q) Inv[q] = b[q];
  return true;
}

// acc + x * y in double for float x, y: the double product of two floats is exact (48 significand
// bits), so one fused multiply-add rounds exactly like the separate multiply and add (half the fp64
// instructions of the normal-equation sums, bit-identical)
LOAM_D double dmac(double acc, float x, float y) { return __builtin_fma((double)x, (double)y, acc); }

// C[m x n] = A[m x k] B[k x n], products and sums in double, one rounding (OpenCV CV_32F gemm)
LOAM_HD void gemm_d(const float* A, const float* B, int m, int k, int n, float* C) {
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int l = 0; l < k; ++l) s += (double)A[i * k + l] * (double)B[l * n + j];
      C[i * n + j] = (float)s;
    }
}

// The iteration-0 degeneracy test (:770-797 odometry, :927-954 mapping) needs the eigenvectors only
// when the smallest eigenvalue cv::eigen reports is below the threshold: otherwise isDegenerate is
// false and matP is never used.  cv::eigen's float Jacobi returns eigenvalues within 2.4 eps_f
// ||A||_inf of the exact ones (measured over 20 000 normal-equation-like matrices,
// tests/test_oracle_components.py::test_jacobi_eigen_error_bound); so when A - (thr + D) I is
// positive definite with D = 2^-14 ||A||_inf (~512 eps_f ||A||_inf), every eigenvalue the Jacobi
// would return is >= thr, and the branch is decided without it.  Positive definiteness: an LDL^T in
// double whose pivots must all be positive (backward error ~1e-15 ||A||, far inside D).  NaN / inf
// entries, and any matrix near the threshold, are not certified: the caller runs the Jacobi.
LOAM_HD bool nondegenerate_certified(const float* A, float thr) {
  double nrm = 0.0;
  for (int i = 0; i < 6; ++i) {
    double rs = 0.0;
    for (int j = 0; j < 6; ++j) rs += fabs((double)A[i * 6 + j]);
    nrm = rs > nrm ? rs : nrm;
  }
  if (!(nrm < 1e30)) return false;
  const double shift = (double)thr + nrm * 0x1p-14;
  double L[6][6], d[6];
  for (int j = 0; j < 6; ++j) {
    double dj = (double)A[j * 6 + j] - shift;
    for (int k = 0; k < j; ++k) dj -= L[j][k] * L[j][k] * d[k];
    if (!(dj > 0.0)) return false;
    d[j] = dj;
    for (int i = j + 1; i < 6; ++i) {
      double v = (double)A[i * 6 + j];
      for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k] * d[k];
      L[i][j] = v / dj;
    }
  }
  return true;
}

// The L-M step on a reduced normal system (shared by odometry :765-826 and mapping :922-974):
// AtA (6x6 float), AtB (6), iteration-0 degeneracy analysis.  One lane.
// ws: >= kLmWs floats of scratch (LDS when called from a kernel lane), iws: >= 12 ints
constexpr int kLmWs = 36 * 6 + 6 + 14 + 6;
// pre_E / pre_V (optional): jacobi<6>(AtA) already computed (jacobi6_wave, by the caller's wave).
// certified: nondegenerate_certified(AtA, eig_thresh) held, so iteration 0 sets isDegenerate = 0
// without the eigen-analysis (matP is left as it was: it is read only when isDegenerate is set)
LOAM_HD void lm_step_tail(const float* AtA_in, int iter, float eig_thresh, int* isDegenerate, float* matP, float* X,
                          float* ws, int* iws, const float* pre_E, const float* pre_V, bool certified);
LOAM_HD void lm_step(const float* AtA_in, const float* AtB_in, int iter, float eig_thresh,
                     int* isDegenerate, float* matP, float* X, float* ws, int* iws,
                     const float* pre_E = nullptr, const float* pre_V = nullptr, bool certified = false) {
  // the QR solve of every iteration works in registers (fully unrolled, constant indices); the
  // iteration-0 analysis (pivoted Jacobi / LU, data-dependent indices) in ws
  float A[36], b[6], qws[14];
  for (int i = 0; i < 36; ++i) A[i] = AtA_in[i];
  for (int i = 0; i < 6; ++i) b[i] = AtB_in[i];
  qr_solve(A, b, 6, 6, X, qws);
  lm_step_tail(AtA_in, iter, eig_thresh, isDegenerate, matP, X, ws, iws, pre_E, pre_V, certified);
}

// qr_solve(A, b, 6, 6, x) by one whole wave (all 64 lanes active), bit-identical to the one-lane
// solve: lane c < 6 holds column c of A in registers, lane 6 holds b.  Per Householder step l the
// column's norm and reflector stay one serial chain (uniform values, as in the one-lane code), but
// the divisions v[i] / nrm and v[i] / v[0] run one per lane, and every column's dot product and
// update (lanes l..5) run at once; b's step l (the one-lane code's second loop, which reads only
// column l's stored reflector and h[l], final after step l) runs on lane 6 beside them.  The back
// substitution is the serial chain on broadcast values.  The one-lane solve was ~1 200 dependent
// instructions (~3 us per L-M step on the streaming path); A (row-major 36) and b are read from
// memory, x is returned to every lane.
LOAM_D bool qr_solve6_wave(const float* A_in, const float* b_in, float (&x)[6]) {
  const int lane = __lane_id();
  const float eps = 1.1920928955078125e-07f * 10;
  const bool isb = lane == 6;
  float col[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) col[i] = lane < 6 ? A_in[i * 6 + (lane < 6 ? lane : 0)] : (isb ? b_in[i] : 0.0f);
#pragma unroll
  for (int l = 0; l < 6; ++l) {
    const int len = 6 - l;
    float s[6];
#pragma unroll
    for (int i = 0; i < len; ++i) s[i] = wl_read(col[l + i], l);
    float nrm = 0.0f;
#pragma unroll
    for (int i = 0; i < len; ++i) nrm += s[i] * s[i];
    const float v0 = s[0];
    s[0] = s[0] + sgn1(s[0]) * sqrtf(nrm);
    nrm = sqrtf(nrm + s[0] * s[0] - v0 * v0);
    float mine = s[0];
#pragma unroll
    for (int i = 1; i < len; ++i)
      if (lane == i) mine = s[i];
    const float myv = mine / nrm;  // lane i: v[i] /= nrm
    float v[6], vp[6];
#pragma unroll
    for (int i = 0; i < len; ++i) v[i] = wl_read(myv, i);
    const float mys = myv / v[0];  // lane i >= 1: the stored A[(l + i) n + l] = v[i] / v[0]
    vp[0] = 1.0f;
#pragma unroll
    for (int i = 1; i < len; ++i) vp[i] = wl_read(mys, i);
    const float h = v[0] * v[0];
    // columns j >= l: dot = sum v[i] A[l + i][j], A -= 2 v[i] dot; b (lane 6, with the stored
    // reflector vp and h[l]): b -= 2 vp[i] dot h
    float dot = 0.0f;
#pragma unroll
    for (int i = 0; i < len; ++i) dot += (isb ? vp[i] : v[i]) * col[l + i];
    if ((lane >= l && lane < 6) || isb) {
#pragma unroll
      for (int i = 0; i < len; ++i) {
        float u = 2 * (isb ? vp[i] : v[i]) * dot;
        if (isb) u = u * h;
        col[l + i] -= u;
      }
    }
    if (lane == l) {
#pragma unroll
      for (int i = 1; i < len; ++i) col[l + i] = vp[i];
    }
  }
  float R[6][6], bb[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    bb[i] = wl_read(col[i], 6);
#pragma unroll
    for (int j = i; j < 6; ++j) R[i][j] = wl_read(col[i], j);
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
#pragma unroll
    for (int j = 5; j > i; --j) bb[i] -= bb[j] * R[i][j];
    if (fabsf(R[i][i]) < eps) {
#pragma unroll
      for (int q = 0; q < 6; ++q) x[q] = 0.0f;
      return false;
    }
    bb[i] /= R[i][i];
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) x[q] = bb[q];
  return true;
}

// lm_step by one whole wave: the QR solve wave-parallel (qr_solve6_wave), the rest on lane 0 (the
// other lanes return; the caller's lane 0 continues with X)
LOAM_D void lm_step_wave(const float* AtA_in, const float* AtB_in, int iter, float eig_thresh, int* isDegenerate,
                         float* matP, float* X, float* ws, int* iws, const float* pre_E = nullptr,
                         const float* pre_V = nullptr, bool certified = false) {
#ifdef LOAM_QR_ONE_LANE  // (experiment builds: the one-lane solve, for A/B)
  if (__lane_id() != 0) return;
  lm_step(AtA_in, AtB_in, iter, eig_thresh, isDegenerate, matP, X, ws, iws, pre_E, pre_V, certified);
  return;
#endif
  float x[6];
  qr_solve6_wave(AtA_in, AtB_in, x);
  if (__lane_id() != 0) return;
#pragma unroll
  for (int q = 0; q < 6; ++q) X[q] = x[q];
  lm_step_tail(AtA_in, iter, eig_thresh, isDegenerate, matP, X, ws, iws, pre_E, pre_V, certified);
}

// lm_step after the QR solve (X holds the solution): the iteration-0 degeneracy analysis and the
// projection of a degenerate step
LOAM_HD void lm_step_tail(const float* AtA_in, int iter, float eig_thresh, int* isDegenerate, float* matP, float* X,
                          float* ws, int* iws, const float* pre_E, const float* pre_V, bool certified) {
  float* A2 = ws + 42;      // 36
  float* V = ws + 78;       // 36
  float* V2 = ws + 114;     // 36
  float* Vi = ws + 150;     // 36
  float* E = ws + 186;      // 6
  float* tmp = ws + 192;    // 36 (LU rhs) / 14 (QR) / 6 (X2)
  if (iter == 0 && certified) {
    *isDegenerate = 0;
  } else if (iter == 0) {
    if (pre_E) {
      for (int i = 0; i < 6; ++i) E[i] = pre_E[i];
      for (int i = 0; i < 36; ++i) V[i] = pre_V[i];
    } else {
      for (int i = 0; i < 36; ++i) A2[i] = AtA_in[i];
      jacobi<6>(A2, E, V, iws);
    }
    for (int i = 0; i < 36; ++i) V2[i] = V[i];
    int degen = 0;
    for (int i = 5; i >= 0; --i) {
      if (E[i] < eig_thresh) {
        for (int j = 0; j < 6; ++j) V2[i * 6 + j] = 0;
        degen = 1;
      } else {
        break;
      }
    }
    *isDegenerate = degen;
    lu_inv6(V, Vi, tmp);
    gemm_d(Vi, V2, 6, 6, 6, matP);
  }
  if (*isDegenerate) {
    for (int i = 0; i < 6; ++i) tmp[i] = X[i];
    gemm_d(matP, tmp, 6, 6, 1, X);
  }
}

LOAM_HD float delta_r(const float* X) {
  double a = loamdev::rad2deg((double)X[0]), b = loamdev::rad2deg((double)X[1]),
         c = loamdev::rad2deg((double)X[2]);
  return (float)sqrt(a * a + b * b + c * c);
}
LOAM_HD float delta_t(const float* X) {
  double a = (double)(X[3] * 100), b = (double)(X[4] * 100), c = (double)(X[5] * 100);
  return (float)sqrt(a * a + b * b + c * c);
}

}  // namespace loamla

#endif
