// Laser mapping on gfx950: the laserMapping loop body (/root/reference/src/laserMapping.cpp:411-1097)
// for P independent map instances (the streaming map, or one per config-4 problem).
//
//  k_mp_prepare    pose prediction (transformAssociateToMap :110-197, fed through the nav_msgs
//                  quaternion round trip :304-321), cube-grid recentring (:440-614) as slot-table
//                  shifts, FOV cube selection (:616-672), FromMap prefix.
//  k_mp_stack      stack to map frame and back (:424-434, :683-691, Q24)
//  vg_run          segmented PCL VoxelGrid (a cascade of hand-written LDS / global radix-sort kernels
//                  by voxel index; equal keys keep input order) for the stacks (:693-701) and the
//                  valid cubes (:1018-1036)
//  k_mp_gather     FromMap = valid cubes concatenated (:674-681), then voxel-hashed (k_hash_build)
//  k_mp_nnfit      one L-M iteration for every instance at once, lane per stack point: the exact
//                  5-NN (:714-719, :821-826) through the 1 m hash (any point within the 1 m acceptance
//                  radius lies in the 27 cells; cells pruned by box distance), the corner PCA with the
//                  3x3 Jacobi / surface 5x3 QR plane (reused while the ordered 5-NN is unchanged),
//                  weight -> accepted row (:721-877), and (fused) the fp64 JᵀJ / Jᵀb partials with
//                  the 6x6 step in the instance's last workgroup (:879-974)
//  k_mp_iter       the step as its own launch (tuning mp_fused_max)
//  k_mp_lm_small / k_mp_lm_stream   the same for a few instances / one (streaming)
//  k_mp_lm_end     transformUpdate (:199-232)
//  k_mp_insert     stack -> cubes in stack order (:980-1016)
//  k_mp_vcopy      per valid cube: old content ++ appended points -> DS input
//  k_mp_compact    new cube store (valid cubes downsampled, others appended) into the other pool
//  k_mp_register   full cloud to the map frame (:1060-1063)

#include <algorithm>
#include <functional>
#include <cstring>
#include <vector>

#include "dev_common.hpp"
#include "mp.hpp"
#include "od.hpp"
#include "pose_math.hpp"

using namespace loamdev;

namespace loam {
#ifdef LOAM_PHASES
__device__ PhaseAcc g_ph_mp = {~0ull, 0ull, 0ull, {{0}}};
#endif


namespace {

constexpr int kMpThreads = 256;

LOAM_D int cube_of(float v, int cen) {  // :446-452, :983-989
  int c = (int)((D(v) + 25.0) / 50.0) + cen;
  if (D(v) + 25.0 < 0) c--;
  return c;
}
LOAM_D int cube_index(int i, int j, int k) { return i + kCubeW * j + kCubeW * kCubeH * k; }

LOAM_D int* slot_table(const MpBuffers& b, int pool, int p) {
  return b.slots + ((size_t)pool * b.P + p) * kCubeNum * 4;
}

// ---------------------------------------------------------------- prepare
// sin / cos of the TobeMapped rotation in double (pointAssociateToMap, :240-257), kept per instance
// in b.rot beside the state: written wherever transformTobeMapped changes (prepare, each L-M
// step, the IMU blend), read by every kernel that maps points.  Per thread they were six double
// sin / cos calls, the larger part of the 5-NN kernel's instructions.
LOAM_D void rot_store(const MpBuffers& b, int p, const float* T) {
  const loampose::MapRot r = loampose::map_rot(T);
  double* d = b.rot + (size_t)p * 6;
  d[0] = r.c0; d[1] = r.s0; d[2] = r.c1; d[3] = r.s1; d[4] = r.c2; d[5] = r.s2;
}
LOAM_D loampose::MapRot rot_load(const MpBuffers& b, int p) {
  const double* d = b.rot + (size_t)p * 6;
  const float* T = b.state + (size_t)p * kMpStateFloats + kMpTobe;
  loampose::MapRot r;
  r.c0 = d[0]; r.s0 = d[1]; r.c1 = d[2]; r.s1 = d[3]; r.c2 = d[4]; r.s2 = d[5];
  r.t3 = T[3]; r.t4 = T[4]; r.t5 = T[5];
  return r;
}

__global__ __launch_bounds__(kMpThreads) void k_mp_prepare(MpBuffers b, MpInput in) {
  const int p = blockIdx.x, tid = threadIdx.x;
  float* st = b.state + (size_t)p * kMpStateFloats;
  int* ist = b.istate + (size_t)p * kMpStateInts;
  int* slots = slot_table(b, b.pool_cur, p);
  __shared__ int sh_shift[3], sh_count[3];
  __shared__ int sh_nshift, sh_c[3], sh_cen[3], sh_scan[16];
  if (tid == 0) {
    float pose[6] = {0, 0, 0, 0, 0, 0};
    if (in.pose)
      for (int k = 0; k < 6; ++k) pose[k] = in.pose[(size_t)p * in.pose_stride + k];
    loampose::pose_through_msg(pose, st + kMpSum);
    loampose::associate_to_map(st + kMpSum, st + kMpBef, st + kMpAft, st + kMpIncre, st + kMpTobe);
    const float* T = st + kMpTobe;
    const loampose::MapRot r = loampose::map_rot(T);
    rot_store(b, p, T);
    const float4 onY = loampose::point_to_map(r, make_float4(0.0f, 10.0f, 0.0f, 0.0f));
    st[kMpOnY] = onY.x; st[kMpOnY + 1] = onY.y; st[kMpOnY + 2] = onY.z;
    int cW = ist[kMiCenW], cH = ist[kMiCenH], cD = ist[kMiCenD];
    int cI = cube_of(T[3], cW), cJ = cube_of(T[4], cH), cK = cube_of(T[5], cD);
    // :454-614: each `while` moves the grid one slab per pass until the centre cube is >= 3 from
    // the edge.  The pass counts are closed-form; a line of cubes shifted by its full length (or
    // more) is entirely cleared, so at most that many slot-table shifts are replayed per axis
    // while the centre indices take every pass (ist[kMiShifts] counts the reference's passes).
    const int dim[3] = {kCubeW, kCubeH, kCubeD};
    int* c[3] = {&cI, &cJ, &cK};
    int* cen[3] = {&cW, &cH, &cD};
    int n = 0;
    long long passes = 0;
    for (int axis = 0; axis < 3; ++axis) {
      long long up = 0, down = 0;
      if (*c[axis] < 3) up = 3 - (long long)*c[axis];
      else if (*c[axis] >= dim[axis] - 3) down = (long long)*c[axis] - (dim[axis] - 4);
      const long long moves = up ? up : down;
      if (moves) {
        *c[axis] += (int)(up - down);
        *cen[axis] += (int)(up - down);
        sh_shift[n] = axis * 2 + (up ? 1 : 0);
        sh_count[n] = (int)(moves < dim[axis] ? moves : dim[axis]);
        ++n;
        passes += moves;
      }
    }
    ist[kMiShifts] = (int)(passes < 0x7fffffff ? passes : 0x7fffffff);
    sh_nshift = n;
    sh_c[0] = cI; sh_c[1] = cJ; sh_c[2] = cK;
    ist[kMiCubeI] = cI; ist[kMiCubeJ] = cJ; ist[kMiCubeK] = cK;
    ist[kMiCenW] = cW; ist[kMiCenH] = cH; ist[kMiCenD] = cD;
    sh_cen[0] = cW; sh_cen[1] = cH; sh_cen[2] = cD;
  }
  __syncthreads();
  for (int s = 0; s < sh_nshift; ++s)
  for (int rep = 0; rep < sh_count[s]; ++rep) {  // slot-table shifts: the cleared cube wraps around
    const int axis = sh_shift[s] >> 1, up = sh_shift[s] & 1;
    const int nAx = axis == 0 ? kCubeW : (axis == 1 ? kCubeH : kCubeD);
    const int na = axis == 0 ? kCubeH : kCubeW, nb = axis == 2 ? kCubeH : kCubeD;
    for (int line = tid; line < na * nb; line += kMpThreads) {
      const int a = line % na, bb = line / na;
      auto at = [&](int c) {
        if (axis == 0) return cube_index(c, a, bb);
        if (axis == 1) return cube_index(a, c, bb);
        return cube_index(a, bb, c);
      };
      int4* sl = (int4*)slots;
      if (up) {
        int4 keep = sl[at(nAx - 1)];
        for (int c = nAx - 1; c >= 1; --c) sl[at(c)] = sl[at(c - 1)];
        keep.y = 0; keep.w = 0;
        sl[at(0)] = keep;
      } else {
        int4 keep = sl[at(0)];
        for (int c = 0; c < nAx - 1; ++c) sl[at(c)] = sl[at(c + 1)];
        keep.y = 0; keep.w = 0;
        sl[at(nAx - 1)] = keep;
      }
    }
    __threadfence_block();  // (one workgroup: the next shift's lines are other threads')
    __syncthreads();
  }
  // FOV selection (:616-672) and FromMap prefix: thread c tests cube c of the 5x5x5
  // neighbourhood (the reference's i, j, k loop order), block scans keep that order
  const float* T = st + kMpTobe;
  const int cI = sh_c[0], cJ = sh_c[1], cK = sh_c[2];
  const int cW = sh_cen[0], cH = sh_cen[1], cD = sh_cen[2];
  bool inFOV = false;
  int ind = 0;
  if (tid < 125) {
    const int i = cI - 2 + tid / 25, j = cJ - 2 + (tid / 5) % 5, k = cK - 2 + tid % 5;
    if (i >= 0 && i < kCubeW && j >= 0 && j < kCubeH && k >= 0 && k < kCubeD) {
      const float ox = st[kMpOnY], oy = st[kMpOnY + 1], oz = st[kMpOnY + 2];
      const float centerX = (float)(50.0 * (i - cW));
      const float centerY = (float)(50.0 * (j - cH));
      const float centerZ = (float)(50.0 * (k - cD));
      for (int ii = -1; ii <= 1; ii += 2)
        for (int jj = -1; jj <= 1; jj += 2)
          for (int kk = -1; kk <= 1; kk += 2) {
            const float cornerX = (float)(D(centerX) + 25.0 * ii);
            const float cornerY = (float)(D(centerY) + 25.0 * jj);
            const float cornerZ = (float)(D(centerZ) + 25.0 * kk);
            const float sq1 = (T[3] - cornerX) * (T[3] - cornerX) + (T[4] - cornerY) * (T[4] - cornerY) +
                              (T[5] - cornerZ) * (T[5] - cornerZ);
            const float sq2 = (ox - cornerX) * (ox - cornerX) + (oy - cornerY) * (oy - cornerY) +
                              (oz - cornerZ) * (oz - cornerZ);
            const float check1 = (float)(100.0 + D(sq1) - D(sq2) - 10.0 * sqrt(3.0) * sqrt(D(sq1)));
            const float check2 = (float)(100.0 + D(sq1) - D(sq2) + 10.0 * sqrt(3.0) * sqrt(D(sq1)));
            if (check1 < 0 && check2 > 0) inFOV = true;
          }
      ind = cube_index(i, j, k);
    }
  }
  const int nC = inFOV ? slots[ind * 4 + 1] : 0, nS = inFOV ? slots[ind * 4 + 3] : 0;
  int nv, accC, accS;
  const int xv = block_excl_scan<kMpThreads>(inFOV ? 1 : 0, sh_scan, nv);
  const int xc = block_excl_scan<kMpThreads>(nC, sh_scan, accC);
  const int xs = block_excl_scan<kMpThreads>(nS, sh_scan, accS);
  int* vp = b.vpre + (size_t)p * (kMaxValid + 1) * 2;
  if (inFOV) {
    b.valid[(size_t)p * kMaxValid + xv] = ind;
    vp[xv * 2 + 0] = xc;
    vp[xv * 2 + 1] = xs;
  }
  if (tid == 0) {
    vp[nv * 2 + 0] = accC;
    vp[nv * 2 + 1] = accS;
    ist[kMiNValid] = nv;
    if (accC + accS > b.map_cap) {
      ist[kMiErr] |= ERR_CAP_MAP;
      accC = accS = 0;
      ist[kMiNValid] = 0;
    }
    b.nfrom[p * 2 + 0] = accC;
    b.nfrom[p * 2 + 1] = accS;
  }
}

// ---------------------------------------------------------------- stacks
__global__ __launch_bounds__(256) void k_mp_stack(MpBuffers b, MpInput in) {
  const int p = blockIdx.y;
  const loampose::MapRot r = rot_load(b, p);
  const int nc = min(in.ncorner[p * in.ncorner_stride], b.capC);
  const int ns = min(in.nsurf[p * in.nsurf_stride], b.capS);
  float4* out = b.stack2 + (size_t)p * b.cap_stack;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nc + ns; i += gridDim.x * 256) {
    const float4 a = i < nc ? in.corner[(size_t)p * in.corner_stride + i]
                            : in.surf[(size_t)p * in.surf_stride + (i - nc)];
    const float4 m = loampose::point_to_map(r, a);
    out[i < nc ? i : b.capC + (i - nc)] = loampose::point_to_tobe_mapped(r, m);
  }
  if (p == 0 && blockIdx.x == 0 && threadIdx.x == 0) { b.vg_cnt[0] = 0; b.vg_cnt[1] = 0; }  // (vg_stack's lists)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const size_t base = (size_t)p * b.cap_stack;
    b.sseg_b[p * 2 + 0] = (int)base;
    b.sseg_e[p * 2 + 0] = (int)base + nc;
    b.sseg_b[p * 2 + 1] = (int)(base + b.capC);
    b.sseg_e[p * 2 + 1] = (int)(base + b.capC) + ns;
    b.sseg_leaf[p * 2 + 0] = 0.2f;
    b.sseg_leaf[p * 2 + 1] = 0.4f;
    if (in.ncorner[p * in.ncorner_stride] > b.capC || in.nsurf[p * in.nsurf_stride] > b.capS)
      b.istate[(size_t)p * kMpStateInts + kMiErr] |= ERR_CAP_STACK;
  }
}

// ---------------------------------------------------------------- segmented VoxelGrid
// PCL VoxelGrid over many segments at once: stacks (2 per instance), valid cubes (2 x
// 125 per instance), the surround map (1).  Per segment: bbox, voxel keys, a stable sort of
// (voxel, position) — the order of PCL's std::sort on (index, point) pairs with equal voxels in
// input order — and one output point per voxel, the float mean of x, y, z, intensity summed in
// sorted order.  vg_run cascades three hand-written kernels by segment size; no library sort.

// The segment's voxel frame (PCL VoxelGrid: bbox over its points, min_b = floor(min / leaf), the
// divb multipliers), or the one the job supplies (j.frame: a split parent's); false when the leaf is
// "too small" for the bbox (PCL then outputs the input unchanged; a supplied frame never is)
template <int NT>
__device__ __forceinline__ bool vg_frame_of(const VgJob& j, int s, const float4* in, int n, float inv, VgFrame& fr) {
  if (j.frame) {
    fr = j.frame[s];
    return true;
  }
  const int tid = threadIdx.x;
  float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
  for (int i = tid; i < n; i += NT) {
    const float4 a = in[i];
    mn[0] = fminf(mn[0], a.x); mn[1] = fminf(mn[1], a.y); mn[2] = fminf(mn[2], a.z);
    mx[0] = fmaxf(mx[0], a.x); mx[1] = fmaxf(mx[1], a.y); mx[2] = fmaxf(mx[2], a.z);
  }
  block_bbox<NT>(mn, mx);
  if (vg_leaf_too_small(mn, mx, inv)) return false;
  fr.m0 = (int)floorf(mn[0] * inv);
  fr.m1 = (int)floorf(mn[1] * inv);
  fr.m2 = (int)floorf(mn[2] * inv);
  fr.divx = (int)floorf(mx[0] * inv) - fr.m0 + 1;
  fr.divy = (int)floorf(mx[1] * inv) - fr.m1 + 1;
  fr.pad = (int)floorf(mx[2] * inv) - fr.m2 + 1;  // (divz: the split's key range)
  return true;
}

// Fused segmented VoxelGrid with an LDS radix sort: one workgroup per segment of at most NT*E
// points does the bbox, the voxel keys, a stable radix sort of (voxel, position) pairs over the
// bits the keys can differ in, and the ordered per-voxel means.  Segments beyond NT*E are appended
// to the job's big list.
template <int NT, int E, int TAG = 0>  // TAG: which VoxelGrid job (vg_run), a distinct symbol for rocprof
__global__ __launch_bounds__(NT) void k_vg_radix(VgJob j) {
  constexpr int N = NT * E;
  __shared__ uint32_t ka[N], kb[N];
  __shared__ uint16_t va[N], vb[N];
  __shared__ uint32_t sc[(NT / 64 + 1) * 8];
  __shared__ int isc[24];
  const int tid = threadIdx.x;
  const int nl = j.list ? *j.list_n : j.nseg;
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    const int s = j.list ? j.list[li] : li;
    if (j.skip && j.skip[s]) continue;  // (written by k_vg_merge; only the cascade's first kernel sees it)
    const int b0 = j.begin[s], b1 = j.end[s], n = b1 - b0;
    if (n <= 0) {
      if (tid == 0) j.out_count[s] = 0;
      continue;
    }
    if (n > N) {
      if (tid == 0) j.big[atomicAdd(j.big_n, 1)] = s;
      continue;
    }
    const float4* in = j.in + b0;
    const float inv = 1.0f / j.leaf[s];
    VgFrame fr;
    if (!vg_frame_of<NT>(j, s, in, n, inv, fr)) {  // "leaf size too small": output = input
      for (int i = tid; i < n; i += NT) j.out[b0 + i] = in[i];
      if (tid == 0) j.out_count[s] = n;
      continue;
    }
    const int m0 = fr.m0, m1 = fr.m1, m2 = fr.m2;
    const uint32_t mul1 = (uint32_t)fr.divx, mul2 = (uint32_t)(fr.divx * fr.divy);
    uint32_t kmax = 0;
    for (int i = tid; i < n; i += NT) {
      const float4 a = in[i];
      const int i0 = (int)(floorf(a.x * inv) - (float)m0);
      const int i1 = (int)(floorf(a.y * inv) - (float)m1);
      const int i2 = (int)(floorf(a.z * inv) - (float)m2);
      const uint32_t key = (uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2;
      ka[i] = key;
      va[i] = (uint16_t)i;
      kmax = key > kmax ? key : kmax;
    }
    kmax = block_max_u32<NT>(kmax >> 1);
    const int nbits = kmax ? 33 - __clz((int)kmax) : (n > 1 ? 1 : 0);  // bits of the max key
    const int cur = block_radix_sort_kv<NT, E>(ka, va, kb, vb, n, nbits, sc);
    const uint32_t* ks = cur ? kb : ka;
    const uint16_t* vs = cur ? vb : va;
    // ordered per-voxel means in one pass: thread t owns sorted positions [t E, t E + E); its E
    // members are gathered at once, each run that starts in the range is summed from its head in
    // sorted order (a run reaching past the range reads on from global memory), and the runs'
    // output slots come from one block scan of the heads per thread
    {
      const int i0 = tid * E;
      uint32_t kk[E];
      float4 a[E];
      int nh = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = i0 + e;
        kk[e] = i < n ? ks[i] : 0u;
        a[e] = i < n ? in[vs[i]] : make_float4(0, 0, 0, 0);
        nh += (i < n && (i == 0 || ks[i - 1] != kk[e])) ? 1 : 0;
      }
      int tot;
      int slot = block_excl_scan<NT>(nh, isc, tot);
      bool open = false;
      uint32_t ck = 0;
      int cstart = 0;
      float sx = 0, sy = 0, sz = 0, si = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = i0 + e;
        if (i < n) {
          const bool head = i == 0 || (e > 0 ? kk[e - 1] != kk[e] : ks[i - 1] != kk[e]);
          if (head) {
            if (open) {
              const float cnt = (float)(i - cstart);
              j.out[b0 + slot++] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
            }
            open = true;
            ck = kk[e];
            cstart = i;
            sx = 0; sy = 0; sz = 0; si = 0;
          }
          if (open) { sx += a[e].x; sy += a[e].y; sz += a[e].z; si += a[e].w; }
        }
      }
      if (open) {
        int m = min(i0 + E, n);  // (the range may end past the segment)
        while (m < n && ks[m] == ck) {
          const float4 b4 = in[vs[m]];
          sx += b4.x; sy += b4.y; sz += b4.z; si += b4.w;
          ++m;
        }
        const float cnt = (float)(m - cstart);
        j.out[b0 + slot] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
      }
      if (tid == 0) j.out_count[s] = tot;
    }
    __syncthreads();  // the LDS arrays are reused by the next segment
  }
}

// The same for segments of up to NT*E = 16384 points with 8 bytes of LDS per point: the voxel
// keys stay in input order (ka[i] = key of point i) and only the 16-bit positions move between
// the two buffers, each radix pass reading its digits through them (tile_rank4 over the whole
// segment); the long surf stacks of VLP-16 sweeps fit it.
// one segment of k_vg_idx with E positions per thread (blocked: thread t owns positions [t E, t E + E)).
// (Round 4: choosing E = 4 / 8 / 16 by segment size, so that a 5k-point stack keeps 625 threads busy
// instead of 313, measured equal at batch 128 and 1024.)
template <int NT, int E>
__device__ __forceinline__ void vg_idx_segment(const VgJob& j, int s, int b0, int n, uint32_t* ka, uint16_t* va, uint16_t* vb,
                           uint32_t* sc, uint32_t* dtot, uint32_t* dbase, float* fsc, int* isc) {
  const int tid = threadIdx.x;
    const float4* in = j.in + b0;
    const float inv = 1.0f / j.leaf[s];
    VgFrame fr;
    if (!vg_frame_of<NT>(j, s, in, n, inv, fr)) {  // "leaf size too small": output = input
      for (int i = tid; i < n; i += NT) j.out[b0 + i] = in[i];
      if (tid == 0) j.out_count[s] = n;
      return;
    }
    const int m0 = fr.m0, m1 = fr.m1, m2 = fr.m2;
    const uint32_t mul1 = (uint32_t)fr.divx, mul2 = (uint32_t)(fr.divx * fr.divy);
    uint32_t kmax = 0;
    for (int i = tid; i < n; i += NT) {
      const float4 a = in[i];
      const int i0 = (int)(floorf(a.x * inv) - (float)m0);
      const int i1 = (int)(floorf(a.y * inv) - (float)m1);
      const int i2 = (int)(floorf(a.z * inv) - (float)m2);
      const uint32_t key = (uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2;
      ka[i] = key;
      va[i] = (uint16_t)i;
      kmax = key > kmax ? key : kmax;
    }
    kmax = block_max_u32<NT>(kmax >> 1);
    const int nbits = kmax ? 33 - __clz((int)kmax) : (n > 1 ? 1 : 0);
    int cur = 0;
    for (int shift = 0; shift < nbits; shift += 4) {
      const uint16_t* vs = cur ? vb : va;
      uint16_t* vd = cur ? va : vb;
      uint32_t k[E];
      uint16_t v[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = tid * E + e;
        v[e] = i < n ? vs[i] : (uint16_t)0;
        k[e] = i < n ? ka[v[e]] : 0u;
      }
      int rank[E];
      tile_rank4<NT, E>(k, shift, n, sc, dtot, rank);
      if (tid == 0) {
        uint32_t r = 0;
        for (int d = 0; d < 16; ++d) { dbase[d] = r; r += dtot[d]; }
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (rank[e] >= 0) vd[dbase[(k[e] >> shift) & 15u] + rank[e]] = v[e];
      __syncthreads();
      cur ^= 1;
    }
    const uint16_t* vs = cur ? vb : va;
    // ordered per-voxel means (as k_vg_radix): thread t owns sorted positions [t E, t E + E),
    // gathered eight at a time
    {
      const int i0 = tid * E;
      int nh = 0;
      uint32_t prev = i0 > 0 && i0 < n ? ka[vs[i0 - 1]] : 0u;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = i0 + e;
        const uint32_t kc = i < n ? ka[vs[i]] : 0u;
        nh += (i < n && (i == 0 || prev != kc)) ? 1 : 0;
        prev = kc;
      }
      int tot;
      int slot = block_excl_scan<NT>(nh, isc, tot);
      bool open = false;
      uint32_t ck = 0;
      int cstart = 0;
      float sx = 0, sy = 0, sz = 0, si = 0;
      prev = i0 > 0 && i0 < n ? ka[vs[i0 - 1]] : 0u;
      constexpr int G = E < 8 ? E : 8;  // gathers in flight (the thread's E positions only)
#pragma unroll
      for (int e0 = 0; e0 < E; e0 += G) {
        float4 a[G];
        uint32_t kk[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int i = i0 + e0 + u;
          kk[u] = i < n ? ka[vs[i]] : 0u;
          a[u] = i < n ? in[vs[i]] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int i = i0 + e0 + u;
          if (i < n) {
            if (i == 0 || prev != kk[u]) {
              if (open) {
                const float cnt = (float)(i - cstart);
                j.out[b0 + slot++] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
              }
              open = true;
              ck = kk[u];
              cstart = i;
              sx = 0; sy = 0; sz = 0; si = 0;
            }
            if (open) { sx += a[u].x; sy += a[u].y; sz += a[u].z; si += a[u].w; }
            prev = kk[u];
          }
        }
      }
      if (open) {
        int m = min(i0 + E, n);
        while (m < n && ka[vs[m]] == ck) {
          const float4 b4 = in[vs[m]];
          sx += b4.x; sy += b4.y; sz += b4.z; si += b4.w;
          ++m;
        }
        const float cnt = (float)(m - cstart);
        j.out[b0 + slot] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
      }
      if (tid == 0) j.out_count[s] = tot;
    }
}

template <int NT, int E, int TAG = 0>  // TAG: which VoxelGrid job (vg_run), a distinct symbol for rocprof
__global__ __launch_bounds__(NT) void k_vg_idx(VgJob j) {
  constexpr int N = NT * E;
  static_assert(N <= 65536, "16-bit positions");
  __shared__ uint32_t ka[N];
  __shared__ uint16_t va[N], vb[N];
  __shared__ uint32_t sc[(NT / 64 + 1) * 8];
  __shared__ uint32_t dtot[16], dbase[16];
  __shared__ float fsc[16];
  __shared__ int isc[24];
  const int tid = threadIdx.x;
  const int nl = j.list ? *j.list_n : j.nseg;
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    const int s = j.list ? j.list[li] : li;
    const int b0 = j.begin[s], b1 = j.end[s], n = b1 - b0;
    if (n <= 0) {
      if (tid == 0) j.out_count[s] = 0;
      continue;
    }
    if (n > N) {
      if (tid == 0) j.big[atomicAdd(j.big_n, 1)] = s;
      continue;
    }
    vg_idx_segment<NT, E>(j, s, b0, n, ka, va, vb, sc, dtot, dbase, fsc, isc);
    __syncthreads();
  }
}

// Segments of any size (those beyond the LDS kernels), one workgroup each, taken from the job's list:
// bbox, voxel keys into the global key array (with the digit histograms of every pass), a stable
// LSD radix sort of (voxel, position) over the key bits through global memory — 4-bit digits, tiles
// of NT*E items ranked in registers (tile_rank4), digit bases carried from tile to tile — and the
// ordered per-voxel means over the sorted arrays.  Rare in VLP-16 batches (long surf stacks); the
// HDL-64E stack and a large surround map take it.
template <int NT, int E, int TAG = 0>  // TAG: which VoxelGrid job (vg_run), a distinct symbol for rocprof
__global__ __launch_bounds__(NT) void k_vg_big(VgJob j) {
  constexpr int TILE = NT * E;
  __shared__ uint32_t hist[8][16];
  __shared__ uint32_t dbase[16], ttot[16];
  __shared__ uint32_t sc[(NT / 64 + 1) * 8];
  __shared__ int isc[24];
  const int tid = threadIdx.x;
  const int nl = *j.list_n;
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    const int s = j.list[li];
    const int b0 = j.begin[s], n = j.end[s] - b0;
    const float4* in = j.in + b0;
    const float inv = 1.0f / j.leaf[s];
    VgFrame fr;
    if (!vg_frame_of<NT>(j, s, in, n, inv, fr)) {  // "leaf size too small": output = input
      for (int i = tid; i < n; i += NT) j.out[b0 + i] = in[i];
      if (tid == 0) j.out_count[s] = n;
      __syncthreads();
      continue;
    }
    const int m0 = fr.m0, m1 = fr.m1, m2 = fr.m2;
    const uint32_t mul1 = (uint32_t)fr.divx, mul2 = (uint32_t)(fr.divx * fr.divy);
    for (int i = tid; i < 8 * 16; i += NT) (&hist[0][0])[i] = 0;
    __syncthreads();
    uint32_t* K = j.keys + b0;
    uint32_t* V = j.vals + b0;
    uint32_t* K2 = j.keys_alt + b0;
    uint32_t* V2 = j.vals_alt + b0;
    uint32_t kmax = 0;
    for (int i = tid; i < n; i += NT) {
      const float4 a = in[i];
      const int i0 = (int)(floorf(a.x * inv) - (float)m0);
      const int i1 = (int)(floorf(a.y * inv) - (float)m1);
      const int i2 = (int)(floorf(a.z * inv) - (float)m2);
      const uint32_t key = (uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2;
      K[i] = key;
      V[i] = (uint32_t)i;
      kmax = key > kmax ? key : kmax;
#pragma unroll
      for (int p = 0; p < 8; ++p) atomicAdd(&hist[p][(key >> (4 * p)) & 15u], 1u);
    }
    kmax = block_max_u32<NT>(kmax >> 1);
    const int nbits = kmax ? 33 - __clz((int)kmax) : (n > 1 ? 1 : 0);
    int cur = 0;  // 0: the data is in (K, V)
    for (int pass = 0; pass * 4 < nbits; ++pass) {
      const uint32_t* ks = cur ? K2 : K;
      const uint32_t* vs = cur ? V2 : V;
      uint32_t* kd = cur ? K : K2;
      uint32_t* vd = cur ? V : V2;
      if (tid == 0) {
        uint32_t r = 0;
        for (int d = 0; d < 16; ++d) { dbase[d] = r; r += hist[pass][d]; }
      }
      __syncthreads();
      for (int t0 = 0; t0 < n; t0 += TILE) {
        const int nt = min(TILE, n - t0);
        uint32_t k[E], v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = tid * E + e;
          k[e] = i < nt ? ks[t0 + i] : 0u;
          v[e] = i < nt ? vs[t0 + i] : 0u;
        }
        int rank[E];
        tile_rank4<NT, E>(k, 4 * pass, nt, sc, ttot, rank);
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (rank[e] >= 0) {
            const int pos = (int)dbase[(k[e] >> (4 * pass)) & 15u] + rank[e];
            kd[pos] = k[e];
            vd[pos] = v[e];
          }
        __syncthreads();
        if (tid < 16) dbase[tid] += ttot[tid];
        __syncthreads();
      }
      cur ^= 1;
    }
    const uint32_t* ks = cur ? K2 : K;
    const uint32_t* vs = cur ? V2 : V;
    // ordered per-voxel means, tile by tile: thread t's E sorted positions, heads counted by one
    // block scan per tile; each head sums its run in sorted order, reading on past its range
    int outn = 0;
    for (int t0 = 0; t0 < n; t0 += TILE) {
      const int i0 = t0 + tid * E;
      uint32_t kk[E];
      int nh = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = i0 + e;
        kk[e] = i < n ? ks[i] : 0u;
        nh += (i < n && (i == 0 || (e > 0 ? kk[e - 1] : ks[i - 1]) != kk[e])) ? 1 : 0;
      }
      int tot;
      int slot = outn + block_excl_scan<NT>(nh, isc, tot);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = i0 + e;
        if (i < n && (i == 0 || (e > 0 ? kk[e - 1] : ks[i - 1]) != kk[e])) {
          float sx = 0, sy = 0, sz = 0, si = 0;
          int m = i;
          while (m < n && ks[m] == kk[e]) {
            const float4 b4 = in[vs[m]];
            sx += b4.x; sy += b4.y; sz += b4.z; si += b4.w;
            ++m;
          }
          const float cnt = (float)(m - i);
          j.out[b0 + slot++] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
        }
      }
      outn += tot;
    }
    if (tid == 0) j.out_count[s] = outn;
    __syncthreads();
  }
}

// The big-segment split (VgSplit, the HDL-64E surf stacks): one workgroup per parent of the job's
// big list computes the parent's frame (vg_frame_of), its voxel keys' top 4 bits (of the bit range
// the frame allows) as a bucket, the bucket sizes, and re-orders the points stably into the buckets
// (tiles ranked in registers by tile_rank4, as k_vg_big's passes): bucket d of parent li becomes
// sub-segment li * 16 + d in the parent's frame.  Equal keys share a bucket and buckets are key
// ranges in order, so the sub-segments' VoxelGrid outputs in bucket order are the parent's output,
// each voxel summed over the same points in the same (input) order.  A parent whose leaf is "too
// small" is copied to its output here (PCL) and gets empty sub-segments; list slots beyond the
// job's big list too.
template <int NT, int E>
__global__ __launch_bounds__(NT) void k_vg_split(VgJob j, VgSplit x) {
  constexpr int TILE = NT * E;
  __shared__ uint32_t sc[(NT / 64 + 1) * 8];
  __shared__ uint32_t hist[16], dbase[16], ttot[16];
  const int tid = threadIdx.x;
  const int nl = min(*j.list_n, x.npar);
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    int* sb = x.begin + (size_t)li * 16;
    int* se = x.end + (size_t)li * 16;
    const int s = j.list[li];
    const int b0 = j.begin[s], n = j.end[s] - b0;
    const float4* in = j.in + b0;
    const float inv = 1.0f / j.leaf[s];
    // the parent's frame (vg_frame_of's, with four loads in flight per thread)
    VgFrame fr;
    {
      float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
      for (int i0 = tid; i0 < n; i0 += 4 * NT) {
        float4 a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = in[min(i0 + u * NT, n - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          mn[0] = fminf(mn[0], a[u].x); mn[1] = fminf(mn[1], a[u].y); mn[2] = fminf(mn[2], a[u].z);
          mx[0] = fmaxf(mx[0], a[u].x); mx[1] = fmaxf(mx[1], a[u].y); mx[2] = fmaxf(mx[2], a[u].z);
        }
      }
      block_bbox<NT>(mn, mx);
      if (vg_leaf_too_small(mn, mx, inv)) {  // "leaf size too small": output = input
        for (int i = tid; i < n; i += NT) j.out[b0 + i] = in[i];
        if (tid == 0) j.out_count[s] = n;
        if (tid < 16) { sb[tid] = 0; se[tid] = 0; }
        __syncthreads();
        continue;
      }
      fr.m0 = (int)floorf(mn[0] * inv);
      fr.m1 = (int)floorf(mn[1] * inv);
      fr.m2 = (int)floorf(mn[2] * inv);
      fr.divx = (int)floorf(mx[0] * inv) - fr.m0 + 1;
      fr.divy = (int)floorf(mx[1] * inv) - fr.m1 + 1;
      fr.pad = (int)floorf(mx[2] * inv) - fr.m2 + 1;
    }
    const uint32_t mul1 = (uint32_t)fr.divx, mul2 = (uint32_t)(fr.divx * fr.divy);
    // the key range the frame allows (keys are uint32: a wider range buckets the wrapped keys by
    // their top bits, still a monotone bucket of the sorted key)
    const uint64_t kmax = (uint64_t)(fr.divx - 1) + (uint64_t)(fr.divy - 1) * (uint64_t)fr.divx +
                          (uint64_t)(fr.pad - 1) * (uint64_t)fr.divx * (uint64_t)fr.divy;
    const uint32_t km = kmax > 0xffffffffull ? 0xffffffffu : (uint32_t)kmax;
    const int bits = km ? 32 - __builtin_clz(km) : 0;
    const int shift = bits > 4 ? bits - 4 : 0;
    auto key_of = [&](const float4& a) {
      const int i0 = (int)(floorf(a.x * inv) - (float)fr.m0);
      const int i1 = (int)(floorf(a.y * inv) - (float)fr.m1);
      const int i2 = (int)(floorf(a.z * inv) - (float)fr.m2);
      return (uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2;
    };
    if (tid < 16) hist[tid] = 0;
    __syncthreads();
    for (int i0 = tid; i0 < n; i0 += 4 * NT) {  // (four loads in flight per thread)
      float4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = in[min(i0 + u * NT, n - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + u * NT < n) atomicAdd(&hist[(key_of(a[u]) >> shift) & 15u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t r = 0;
      for (int d = 0; d < 16; ++d) { dbase[d] = r; r += hist[d]; }
    }
    __syncthreads();
    if (tid < 16) {  // the sub-segments; the non-empty ones listed for the cascade
      const int k = li * 16 + tid;
      sb[tid] = b0 + (int)dbase[tid];
      se[tid] = b0 + (int)(dbase[tid] + hist[tid]);
      x.leaf[k] = j.leaf[s];
      x.frame[k] = fr;
      x.out_count[k] = 0;
      if (hist[tid]) x.ilist[atomicAdd(&x.counts[2], 1)] = k;
    }
    float4* dst = x.pts + b0;
    for (int t0 = 0; t0 < n; t0 += TILE) {
      const int nt = min(TILE, n - t0);
      uint32_t k[E];
      float4 a[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = tid * E + e;
        a[e] = i < nt ? in[t0 + i] : make_float4(0, 0, 0, 0);
        k[e] = i < nt ? key_of(a[e]) : 0u;
      }
      int rank[E];
      tile_rank4<NT, E>(k, shift, nt, sc, ttot, rank);
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (rank[e] >= 0) dst[dbase[(k[e] >> shift) & 15u] + rank[e]] = a[e];
      __syncthreads();
      if (tid < 16) dbase[tid] += ttot[tid];
      __syncthreads();
    }
  }
}

// the split parents' outputs: the 16 sub-segments' VoxelGrid outputs concatenated in bucket order
// into the parent's output (one workgroup per parent)
template <int NT>
__global__ __launch_bounds__(NT) void k_vg_join(VgJob j, VgSplit x) {
  __shared__ int pre[17];
  const int tid = threadIdx.x;
  const int nl = min(*j.list_n, x.npar);
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    const int s = j.list[li];
    const int* sb = x.begin + (size_t)li * 16;
    const int* se = x.end + (size_t)li * 16;
    const int* sc = x.out_count + (size_t)li * 16;
    if (tid == 0) {
      int r = 0, any = 0;
      for (int d = 0; d < 16; ++d) {
        pre[d] = r;
        const int m = se[d] - sb[d];
        any |= m;
        r += m > 0 ? sc[d] : 0;
      }
      pre[16] = any ? r : -1;  // (-1: the parent was copied by k_vg_split)
    }
    __syncthreads();
    if (pre[16] >= 0) {  // output t of the parent: bucket d = the last with pre[d] <= t
      const int b0 = j.begin[s], tot = pre[16];
      for (int t0 = tid; t0 < tot; t0 += 4 * NT) {
        float4 v[4];
        int o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int t = t0 + u * NT;
          int d = 0;
#pragma unroll
          for (int step = 8; step > 0; step >>= 1)
            if (d + step < 16 && pre[d + step] <= t) d += step;
          o[u] = t;
          v[u] = t < tot ? x.out[sb[d] + (t - pre[d])] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (o[u] < tot) j.out[b0 + o[u]] = v[u];
      }
      if (tid == 0) j.out_count[s] = tot;
    }
    __syncthreads();
  }
}

// Incremental VoxelGrid of a cube segment (:1018-1036) whose first nold points are the cube's
// previous VoxelGrid output and whose tail is this frame's appended points.  A VoxelGrid output
// lists one point per voxel in voxel order; when the old points' voxel keys (under this segment's
// bounding box: the order of absolute grid cells (k, j, i) does not depend on it) are strictly
// increasing, the stable (voxel, position) sort of the whole segment is the merge of the old points
// with the sorted tail, old first within a voxel (they precede the tail in input order).  So only the
// tail is sorted (LDS bitonic, <= NEW points), and each output voxel sums its members in input
// order: its old point, then its tail points — the same float sums as the full sort.  Segments whose
// old keys are not strictly increasing (a cube appended to without a VoxelGrid since, or a mean
// rounded into a neighbouring voxel), whose keys exceed the cascade's 24 sorted bits, or whose box
// is "too small" are left to the cascade (skip[s] = 0).
// (segments beyond the cascade's LDS tiers, which k_vg_big would sort through global memory; the
// LDS tiers measured faster than the merge on 2k-12k segments)
// (Tuning::vg_merge_min: 12288 by default, the largest LDS tier)
constexpr int kVgMergeNew = 8192;
template <int NT, int NEW>
__global__ __launch_bounds__(NT) void k_vg_merge(VgJob j) {
  static_assert((NEW & (NEW - 1)) == 0 && NEW % NT == 0 && NEW <= 65536, "bitonic sort / scan layout");
  __shared__ uint64_t nk[NEW];      // tail (key << 32 | tail position), sorted
  __shared__ uint16_t nhp[NEW];     // first entry in nk of each tail voxel that holds no old point
  __shared__ int isc[24];
  const int tid = threadIdx.x;
  const int nl = *j.mlist_n;
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    const int s = j.mlist[li];
    const int b0 = j.begin[s], n = j.end[s] - b0, nold = j.nold[s], nnew = n - nold;
    const float4* in = j.in + b0;
    float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (int i = tid; i < n; i += NT) {
      const float4 a = in[i];
      mn[0] = fminf(mn[0], a.x); mn[1] = fminf(mn[1], a.y); mn[2] = fminf(mn[2], a.z);
      mx[0] = fmaxf(mx[0], a.x); mx[1] = fmaxf(mx[1], a.y); mx[2] = fmaxf(mx[2], a.z);
    }
    block_bbox<NT>(mn, mx);
    const float inv = 1.0f / j.leaf[s];
    if (vg_leaf_too_small(mn, mx, inv)) {  // (the cascade copies it)
      if (tid == 0) j.skip[s] = 0;
      continue;
    }
    const int m0 = (int)floorf(mn[0] * inv), m1 = (int)floorf(mn[1] * inv), m2 = (int)floorf(mn[2] * inv);
    const int divx = (int)floorf(mx[0] * inv) - m0 + 1, divy = (int)floorf(mx[1] * inv) - m1 + 1;
    const uint32_t mul1 = (uint32_t)divx, mul2 = (uint32_t)(divx * divy);
    auto key_of = [&](const float4& a) {
      const int i0 = (int)(floorf(a.x * inv) - (float)m0);
      const int i1 = (int)(floorf(a.y * inv) - (float)m1);
      const int i2 = (int)(floorf(a.z * inv) - (float)m2);
      return (uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2;
    };
    // the old keys (global scratch, the segment's range of the sort arrays) and their order check
    uint32_t* K = j.keys + b0;
    bool bad = false;
    for (int i = tid; i < nold; i += NT) {
      const uint32_t k = key_of(in[i]);
      K[i] = k;
      bad |= k >= (1u << 24);
    }
    // the tail's (key, position), padded to a power of two for the sort
    int P2 = 1;
    while (P2 < nnew) P2 <<= 1;
    for (int t = tid; t < P2; t += NT) {
      uint64_t e = ~0ull;
      if (t < nnew) {
        const uint32_t k = key_of(in[nold + t]);
        bad |= k >= (1u << 24);
        e = ((uint64_t)k << 32) | (uint32_t)t;
      }
      nk[t] = e;
    }
    __syncthreads();
    for (int i = tid + 1; i < nold; i += NT) bad |= K[i] <= K[i - 1];
    if (__syncthreads_or(bad)) {
      if (tid == 0) j.skip[s] = 0;
      continue;
    }
    if (P2 > 1) block_bitonic_sort<NT>(nk, P2);
    __syncthreads();
    // lower_bound of key k in the old keys (global, ascending)
    auto old_lb = [&](uint32_t k) {
      int lo = 0, hi = nold;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (K[mid] < k) lo = mid + 1; else hi = mid;
      }
      return lo;
    };
    // the tail's voxels that hold no old point, compacted in key order (NEW / NT entries per thread)
    constexpr int PT = NEW / NT;
    int fl[PT], cntf = 0;
#pragma unroll
    for (int u = 0; u < PT; ++u) {
      const int t = tid * PT + u;
      fl[u] = 0;
      if (t < nnew) {
        const uint32_t k = (uint32_t)(nk[t] >> 32);
        if (t == 0 || (uint32_t)(nk[t - 1] >> 32) != k) {
          const int at = old_lb(k);
          fl[u] = (at == nold || K[at] != k) ? 1 : 0;
        }
      }
      cntf += fl[u];
    }
    int m = 0;
    int r = block_excl_scan<NT>(cntf, isc, m);
#pragma unroll
    for (int u = 0; u < PT; ++u)
      if (fl[u]) {
        const int t = tid * PT + u;
        nhp[r] = (uint16_t)t;
        ++r;
      }
    __syncthreads();
    // sums of a voxel's tail members from tail entry e on (sorted: input order within the voxel)
    auto add_tail = [&](int e, uint32_t k, float& sx, float& sy, float& sz, float& si, int& c) {
      for (; e < nnew && (uint32_t)(nk[e] >> 32) == k; ++e) {
        const float4 a = in[nold + (int)(uint32_t)nk[e]];
        sx += a.x; sy += a.y; sz += a.z; si += a.w;
        ++c;
      }
    };
    // old voxels: slot = i + (tail-only voxels before it); members = the old point, then its tail run
    for (int i = tid; i < nold; i += NT) {
      const uint32_t k = K[i];
      int lo = 0, hi = m;  // tail-only voxels with a smaller key
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((uint32_t)(nk[nhp[mid]] >> 32) < k) lo = mid + 1; else hi = mid;
      }
      const int slot = i + lo;
      int e0 = 0, e1 = nnew;  // first tail entry with key >= k
      while (e0 < e1) {
        const int mid = (e0 + e1) >> 1;
        if ((uint32_t)(nk[mid] >> 32) < k) e0 = mid + 1; else e1 = mid;
      }
      const float4 a = in[i];
      float sx = 0, sy = 0, sz = 0, si = 0;
      sx += a.x; sy += a.y; sz += a.z; si += a.w;
      int c = 1;
      add_tail(e0, k, sx, sy, sz, si, c);
      const float cnt = (float)c;
      j.out[b0 + slot] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
    }
    // tail-only voxels: slot = r + (old voxels before it)
    for (int q = tid; q < m; q += NT) {
      const uint32_t k = (uint32_t)(nk[nhp[q]] >> 32);
      const int slot = q + old_lb(k);
      float sx = 0, sy = 0, sz = 0, si = 0;
      int c = 0;
      add_tail(nhp[q], k, sx, sy, sz, si, c);
      const float cnt = (float)c;
      j.out[b0 + slot] = make_float4(sx / cnt, sy / cnt, sz / cnt, si / cnt);
    }
    if (tid == 0) {
      j.out_count[s] = nold + m;
      j.skip[s] = 1;
    }
    __syncthreads();
  }
}

// The cascade: the fused LDS kernel at cap1 points (2048: 256 threads, for the many small cube
// segments; 12288: 1024 threads) over every segment; the segments beyond it through the 12288
// kernel (after the 2048 one), then the rest through k_vg_big.  The list-driven launches use fixed
// grids whose workgroups leave at once when their lists are short.  finish = false: the caller
// knows every segment fits cap1 (streaming stacks), only the first launch is enqueued.
// tier2_idx: the second tier is k_vg_idx (16384 points; the long surf stacks) rather than
// k_vg_radix<1024, 12> (12288; measured faster on the 2k-12k cube segments: at batch 1024 the cubes
// took 0.68 ms/step with it against 0.85 with k_vg_idx, the stacks 0.86 with k_vg_idx against 1.20)
// TAG: kVgStack / kVgCubes / kVgSurround, so a kernel trace or PMC pass tells the jobs apart
constexpr int kVgListGrid = 1024, kVgBigGrid = 256;
constexpr int kVgStack = 0, kVgCubes = 1, kVgSurround = 2;
// split (the stack job's VgSplit, when it holds every segment of the job as a parent): the segments
// the cascade's LDS kernels cannot take are split into key-range buckets (k_vg_split / k_vg_join)
// instead of k_vg_big; split_early: already the segments beyond the first kernel (instead of the
// second tier too)
template <int TAG>
hipError_t vg_run(const VgJob& j0, hipStream_t st, int cap1, bool finish = true, bool tier2_idx = false,
                  const VgSplit* split = nullptr, bool split_early = false) {
  if (j0.nseg == 0) return hipSuccess;
  if (!j0.zeroed) {
    const hipError_t e = hipMemsetAsync(j0.counts, 0, 2 * sizeof(int), st);
    if (e != hipSuccess) return e;
  }
  if (split && split->npar < j0.nseg) split = nullptr;
  // the segments of list `l` (count at j0.counts + l) through the split: 16 key-range buckets each,
  // the buckets through the cascade in their parent's frame, the outputs joined
  auto run_split = [&](int l) -> hipError_t {
    VgJob c = j0;
    c.list = j0.lists[l];
    c.list_n = j0.counts + l;
    const hipError_t ez = hipMemsetAsync(split->counts, 0, 3 * sizeof(int), st);
    if (ez != hipSuccess) return ez;
    hipLaunchKernelGGL((k_vg_split<1024, 12>), dim3(std::min(split->npar, 256)), dim3(1024), 0, st, c, *split);
    VgJob sj = j0;
    sj.in = split->pts;
    sj.out = split->out;
    sj.begin = split->begin;
    sj.end = split->end;
    sj.leaf = split->leaf;
    sj.out_count = split->out_count;
    sj.frame = split->frame;
    sj.nseg = split->npar * 16;
    sj.lists[0] = split->lists[0];
    sj.lists[1] = split->lists[1];
    sj.counts = split->counts;
    sj.zeroed = true;                  // (counts[0..1] zeroed above)
    sj.list = split->ilist;            // the non-empty sub-segments k_vg_split listed
    sj.list_n = split->counts + 2;
    sj.grid_max = 2048;                // (the list is empty unless the job had big segments)
    const hipError_t e = vg_run<TAG>(sj, st, 2048, true, true);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_vg_join<1024>), dim3(std::min(split->npar, 256)), dim3(1024), 0, st, c, *split);
    return hipGetLastError();
  };
  // the caller's input list (non-empty segments) is walked by a fixed grid
  const int grid = std::min(j0.grid_max, j0.list ? std::min(j0.nseg, 8192) : std::min(j0.nseg, 65536));
  VgJob a = j0;
  a.big = j0.lists[0];
  a.big_n = j0.counts;
  int last = 0;  // the list k_vg_big takes
  if (cap1 <= 2048) {
    hipLaunchKernelGGL((k_vg_radix<256, 8, TAG>), dim3(grid), dim3(256), 0, st, a);
    if (finish && split && split_early) return run_split(0);
    if (finish) {
      VgJob b = j0;
      b.list = j0.lists[0];
      b.list_n = j0.counts;
      b.big = j0.lists[1];
      b.big_n = j0.counts + 1;
      if (tier2_idx) hipLaunchKernelGGL((k_vg_idx<1024, 16, TAG>), dim3(std::min(j0.nseg, kVgListGrid)), dim3(1024), 0, st, b);
      else hipLaunchKernelGGL((k_vg_radix<1024, 12, TAG>), dim3(std::min(j0.nseg, kVgListGrid)), dim3(1024), 0, st, b);
      last = 1;
    }
  } else {
    hipLaunchKernelGGL((k_vg_radix<1024, 12, TAG>), dim3(grid), dim3(1024), 0, st, a);
  }
  if (finish) {
    if (split) return run_split(last);
    VgJob c = j0;
    c.list = j0.lists[last];
    c.list_n = j0.counts + last;
    hipLaunchKernelGGL((k_vg_big<1024, 12, TAG>), dim3(std::min(j0.nseg, kVgBigGrid)), dim3(1024), 0, st, c);
  }
  return hipGetLastError();
}

// the instance buffers' VoxelGrid scratch (sort arrays, cascade lists)
VgJob vg_job(const MpBuffers& b) {
  VgJob j;
  j.keys = b.vg_k; j.keys_alt = b.vg_k2; j.vals = b.vg_v; j.vals_alt = b.vg_v2;
  j.lists[0] = b.vg_l0; j.lists[1] = b.vg_l1; j.counts = b.vg_cnt;
  return j;
}

// ---------------------------------------------------------------- FromMap gather
__global__ __launch_bounds__(256) void k_mp_gather(MpBuffers b) {
  const int p = blockIdx.y;
  const int nv = b.istate[(size_t)p * kMpStateInts + kMiNValid];
  const int* vp = b.vpre + (size_t)p * (kMaxValid + 1) * 2;
  const int* slots = slot_table(b, b.pool_cur, p);
  const float4* pool = b.pool + ((size_t)b.pool_cur * b.P + p) * b.map_cap;
  const int totC = vp[nv * 2 + 0], totS = vp[nv * 2 + 1];
  float4* out = b.from + (size_t)p * b.map_cap;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < totC + totS; i += gridDim.x * 256) {
    const int kind = i < totC ? 0 : 1;
    const int t = kind ? i - totC : i;
    int lo = 0, hi = nv - 1;   // last valid cube with prefix <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (vp[mid * 2 + kind] <= t) lo = mid; else hi = mid - 1;
    }
    const int ind = b.valid[(size_t)p * kMaxValid + lo];
    out[i] = pool[slots[ind * 4 + 2 * kind] + (t - vp[lo * 2 + kind])];
  }
}

// ---------------------------------------------------------------- L-M
struct Top5 {
  float d[5];
  int i[5];
};
// (distance, index) as one ordered 64-bit key: distances are >= +0, so their bits order as they do
LOAM_D uint64_t top5_key(float d, int idx) { return ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)idx; }
// sorted insertion of a key below K_4 (branch-free: lt_k = key < K_k is monotone in k, so slot k
// takes K_{k-1} where lt_{k-1}, the key where lt_k alone, else keeps K_k)
LOAM_D void top5_insert(Top5& t, const uint64_t (&K)[5], uint64_t key) {
  const bool l0 = key < K[0], l1 = key < K[1], l2 = key < K[2], l3 = key < K[3];
  const uint64_t N[5] = {l0 ? key : K[0], l0 ? K[0] : (l1 ? key : K[1]), l1 ? K[1] : (l2 ? key : K[2]),
                         l2 ? K[2] : (l3 ? key : K[3]), l3 ? K[3] : key};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    t.d[k] = __uint_as_float((uint32_t)(N[k] >> 32));
    t.i[k] = (int)(uint32_t)N[k];
  }
}
// an offer that cannot repeat a held point (the 5-NN candidate walk: every map point is listed
// once, and a list seeded with copies of the bound B takes only keys below B)
LOAM_D void top5_offer_new(Top5& t, float d, int idx) {
  const uint64_t key = top5_key(d, idx);
  uint64_t K[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) K[k] = top5_key(t.d[k], t.i[k]);
  if (key < K[4]) top5_insert(t, K, key);
}
LOAM_D void top5_offer(Top5& t, float d, int idx) {
  // ascending (distance, index); a point already held is skipped (the merge of lists)
  const uint64_t key = top5_key(d, idx);
  uint64_t K[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) K[k] = top5_key(t.d[k], t.i[k]);
  if (key < K[4] && key != K[0] && key != K[1] && key != K[2] && key != K[3]) top5_insert(t, K, key);
}

// the 27 neighbour cells (index (dx+1) + 3(dy+1) + 9(dz+1)): centre, faces, edges, corners
__constant__ int kCellOrder[27] = {13, 4, 10, 12, 14, 16, 22, 1, 3, 5, 7, 9, 11, 15, 17, 19, 21, 23, 25,
                                   0, 2, 6, 8, 18, 20, 24, 26};

// exact 5-NN within the 27 cells around q (1 m cells), as far as it matters: visited centre,
// faces, edges, corners; a cell is skipped when its box distance exceeds the current 5th
// distance or reaches the 1 m acceptance radius (the caller rejects a 5th neighbour at >= 1 m).
// Box distances are lower bounds of the float squared distances (monotone rounding of the same
// expression), so every neighbour that can be accepted is found exactly.
// t may arrive seeded with real map points (their distances to q): they bound the search from
// the start and do not change the result.
// work: candidates evaluated + (bucket ranges read << kWorkCellShift), summed per lane
constexpr int kWorkCellShift = 21;
LOAM_D void knn5(const int* start, const float4* hp, int T, float4 q, Top5& t, int& work) {
  if (T <= 0) return;
  const int cx = cell_of(q.x, 1.0f), cy = cell_of(q.y, 1.0f), cz = cell_of(q.z, 1.0f);
  const float gxl = q.x - (float)cx, gyl = q.y - (float)cy, gzl = q.z - (float)cz;
  const float gxh = (float)(cx + 1) - q.x, gyh = (float)(cy + 1) - q.y, gzh = (float)(cz + 1) - q.z;
#pragma unroll 1
  for (int o = 0; o < 27; ++o) {
    const int c = kCellOrder[o];
    const int dx = c % 3 - 1, dy = (c / 3) % 3 - 1, dz = c / 9 - 1;
    const float gx = dx < 0 ? gxl : (dx > 0 ? gxh : 0.0f);
    const float gy = dy < 0 ? gyl : (dy > 0 ? gyh : 0.0f);
    const float gz = dz < 0 ? gzl : (dz > 0 ? gzh : 0.0f);
    const float bd = sqdist(gx, gy, gz, 0.0f, 0.0f, 0.0f);
    if (bd >= 1.0f || bd > t.d[4]) continue;
    const uint32_t h = cell_hash(cx + dx, cy + dy, cz + dz) & (uint32_t)(T - 1);
    const int b0 = start[h], b1 = start[h + 1];
    work += (b1 - b0) + (1 << kWorkCellShift);
    // four independent loads in flight per step: the loop is bound by gather latency
    for (int k = b0; k < b1; k += 4) {
      float4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = hp[min(k + u, b1 - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k + u < b1) top5_offer(t, sqdist(a[u].x, a[u].y, a[u].z, q.x, q.y, q.z), __builtin_bit_cast(int, a[u].w));
    }
  }
}

// batch-size launch choices (k_mp_lm_small, k_mp_nnfit<true> or + k_mp_iter): the context's Tuning
// (engine.hpp), MpBuffers::tune
constexpr int kMpQueryThreads = 256;
// lanes per query in k_mp_lm_small (streaming: the per-query search chain is the latency)
#ifndef LOAM_MP_NN_LANES
#define LOAM_MP_NN_LANES 8  // (config 3 sequential ms/sweep: 1 -> 0.972, 2 -> 1.009, 4 -> 0.943, 8 -> 0.933)
#endif
constexpr int kMpNnLanes = LOAM_MP_NN_LANES;
// k_mp_nnfit workgroup size: one wave (round 3's fit kernel, ms/step at batch 1024: 256 -> 1.27-1.29,
// 128 -> 1.16-1.20, 64 -> 1.17)
constexpr int kMpFitThreads = 64;

// The same search with the lane's work flattened: first every cell the lane may need (box
// distance below 1 m and not above the seeded 5th distance) is listed with its bucket range — 27
// independent loads in flight — then one loop runs over the concatenated candidates, so a wave
// iterates max(candidates per lane) instead of the union of its lanes' cells x buckets.  `lst` =
// the lane's LDS column (stride kMpQueryThreads).  Ranges are packed start:19 | count:13; a lane
// whose ranges do not fit falls back to knn5.
#ifndef LOAM_NN_INFLIGHT
#define LOAM_NN_INFLIGHT 8  // measured k_mp_nn ms/step: 2 -> 4.17, 4 -> 3.95, 8 -> 3.88, 16 -> 5.33
#endif
constexpr int kNnInFlight = LOAM_NN_INFLIGHT;
#ifndef LOAM_NN_LIST
#define LOAM_NN_LIST 27  // k_mp_nn list entries per lane (non-empty cells beyond it: the unlisted search)
#endif
constexpr int kNnListCap = LOAM_NN_LIST;
// cells whose bucket-range loads are in flight together
#ifndef LOAM_NN_RANGE_GROUP
#define LOAM_NN_RANGE_GROUP 27  // one-word records: all 27 in flight (ms/step: 9 -> 3.11, 27 -> 3.04; 8-byte pairs: 1 -> 3.83, 9 -> 3.51)
#endif
constexpr int kNnRangeGroup = LOAM_NN_RANGE_GROUP;
// L > 1: one of L lanes searching the same query: every lane lists the same cells, lane `sub`
// takes the candidates sub, sub + L, ... of the concatenated list (a crowded cell is shared too);
// the caller merges the L partial top-5 lists (knn5_merge)
template <int S = kMpQueryThreads, int L = 1, int CAPL = 27>
LOAM_D void knn5_flat(const int* start, const uint32_t* rec, const float4* hp, int T, float4 q, Top5& t,
                      uint32_t* lst, int& work, int sub = 0) {
  if (T <= 0) return;
  const int cx = cell_of(q.x, 1.0f), cy = cell_of(q.y, 1.0f), cz = cell_of(q.z, 1.0f);
  const float gxl = q.x - (float)cx, gyl = q.y - (float)cy, gzl = q.z - (float)cz;
  const float gxh = (float)(cx + 1) - q.x, gyh = (float)(cy + 1) - q.y, gzh = (float)(cz + 1) - q.z;
  const float bound = t.d[4];
  int n = 0, total = 0;
  bool fits = true;
  // the range loads of a group of cells are all issued before any is used (a load whose count is
  // tested in the same block is waited for at once: one dependent round trip per cell)
#pragma unroll
  for (int g0 = 0; g0 < 27; g0 += kNnRangeGroup) {
    uint32_t rg[kNnRangeGroup];
#pragma unroll
    for (int u = 0; u < kNnRangeGroup; ++u) {
      const int o = g0 + u;
      if (o >= 27) break;
      const int c = kCellOrder[o];
      const int dx = c % 3 - 1, dy = (c / 3) % 3 - 1, dz = c / 9 - 1;
      const float gx = dx < 0 ? gxl : (dx > 0 ? gxh : 0.0f);
      const float gy = dy < 0 ? gyl : (dy > 0 ? gyh : 0.0f);
      const float gz = dz < 0 ? gzl : (dz > 0 ? gzh : 0.0f);
      const float bd = sqdist(gx, gy, gz, 0.0f, 0.0f, 0.0f);
      rg[u] = 0;
      if (bd < 1.0f && bd <= bound) {
        const uint32_t h = cell_hash(cx + dx, cy + dy, cz + dz) & (uint32_t)(T - 1);
        rg[u] = rec[h];  // the bucket's range packed in one word (hash_rec)
      }
    }
#pragma unroll
    for (int u = 0; u < kNnRangeGroup; ++u) {
      if (g0 + u >= 27) break;
      const uint32_t e = rg[u];
      if (e == kRecNone) fits = false;
      else if (e >> 19) {
        if (n < CAPL) {
          lst[n * S] = e;
          ++n;
          total += (int)(e >> 19);
        } else {
          fits = false;  // more non-empty cells than the list holds
        }
      }
    }
  }
  if (!fits) {
    knn5(start, hp, T, q, t, work);
    return;
  }
  work += total + (n << kWorkCellShift);
  // the list is walked one entry ahead: the LDS read of the next entry is issued when the current
  // one is taken, so its latency is not on the candidate chain
  int ci = 1, left = 0, pos = 0;
  uint32_t nx = lst[0];
  auto take = [&]() {
    pos = (int)(nx & ((1u << 19) - 1));
    left = (int)(nx >> 19);
    nx = lst[min(ci, CAPL - 1) * S];
    ++ci;
  };
  auto next = [&]() {  // index of the lane's next candidate
    if (left == 0) take();
    --left;
    return pos++;
  };
  auto skip = [&](int m) {  // pass over m candidates (the other lanes' share)
    while (m > 0) {
      if (left == 0) take();
      const int s = min(m, left);
      pos += s;
      left -= s;
      m -= s;
    }
  };
  const int mine = L == 1 ? total : (total > sub ? (total - sub + L - 1) / L : 0);
  if (L > 1 && mine > 0) skip(sub);  // (mine > 0: the list holds more than sub candidates)
  for (int k = 0; k < mine; k += kNnInFlight) {  // independent gathers in flight per step
    int idx[kNnInFlight];
#pragma unroll
    for (int u = 0; u < kNnInFlight; ++u) {
      if (k + u < mine) {
        idx[u] = next();
        if (L > 1 && k + u + 1 < mine) skip(L - 1);
      } else {
        idx[u] = idx[0];
      }
    }
#ifdef LOAM_BOUNDS_CHECK
    for (int u = 0; u < kNnInFlight; ++u) LOAM_CHECK(idx[u] >= 0 && idx[u] < (1 << 19) + (1 << 13), idx[u], total);
#endif
    float4 a[kNnInFlight];
#pragma unroll
    for (int u = 0; u < kNnInFlight; ++u) a[u] = hp[idx[u]];
#pragma unroll
    for (int u = 0; u < kNnInFlight; ++u)
      if (k + u < mine) top5_offer_new(t, sqdist(a[u].x, a[u].y, a[u].z, q.x, q.y, q.z), __builtin_bit_cast(int, a[u].w));
  }
}

// the L lanes of a query group (aligned, consecutive) exchange their top-5 lists in log2(L)
// butterfly rounds; top5_offer keeps the 5 smallest (distance, index) of the union without
// duplicates, which does not depend on the order of the offers, so every lane of the group ends
// with the list a single lane's search over all the cells would have found
template <int L>
LOAM_D void knn5_merge(Top5& t) {
#pragma unroll
  for (int m = 1; m < L; m <<= 1) {
    float od[5];
    int oi[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      od[k] = __shfl_xor(t.d[k], m, 64);
      oi[k] = __shfl_xor(t.i[k], m, 64);
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
      if (oi[k] != 0x7fffffff) top5_offer(t, od[k], oi[k]);
  }
}


}  // namespace

__global__ void k_mp_lm_begin(MpBuffers b) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= b.P) return;
  int* ist = b.istate + (size_t)p * kMpStateInts;
  const int nfc = b.nfrom[p * 2 + 0], nfs = b.nfrom[p * 2 + 1];
  ist[kMiStackC] = b.sseg_cnt[p * 2 + 0];
  ist[kMiStackS] = b.sseg_cnt[p * 2 + 1];
  ist[kMiFromC] = nfc;
  ist[kMiFromS] = nfs;
  ist[kMiLmRan] = (nfc > 10 && nfs > 100) ? 1 : 0;  // :706
  ist[kMiStop] = 0;
  ist[kMiIters] = 0;
  ist[kMiRows] = 0;
  ist[kMiFits] = 0;
  ist[kMiDegSteps] = 0;
  ist[kMiNnCand] = 0;
  ist[kMiNnCells] = 0;
  if (p == 0 && b.P == 1) ++b.ls_epoch[0];  // (k_mp_lm_stream's publication words)
}

// One L-M iteration's correspondences (:714-877), lane per stack point (corner, then surf), in
// per-query pieces shared by the batch kernel (k_mp_nnfit) and the small-batch / streaming kernels
// (k_mp_lm_small, k_mp_lm_stream).
//   mp_nn_query   the point at the current TobeMapped pose and its exact 5-NN (seeded with the
//                 previous iteration's), stored in q_nn
//   mp_fit_query  the line (corner PCA, 3x3 Jacobi) or plane (5x3 QR) through the 5 neighbours and
//                 the weighted residual.  A fit depends on nothing but the ordered 5 neighbours, so
//                 it is kept per query and reused while the ordered 5-NN is unchanged from the
//                 previous iteration (bit-identical to refitting)
//   mp_row_accum  the accepted row's J (:897-921) added in fp64
//   mp_step       the 6x6 step on the summed normal equations (:922-974)
namespace {
// the ordered 5-NN a fit was made for, and the fit: corner (x1, y1, z1, valid), (x2, y2, z2, -);
// surf (pa, pb, pc, pd), (valid, -, -, -)
struct MpFit {
  int4 n0, n1;
  float4 g0, g1;
};

// an instance's search inputs, resolved once per workgroup
struct MpNnCtx {
  const float4* stack;
  const int *hcs, *hss;
  const uint32_t *hcr, *hsr;
  const float4 *hcp, *hsp, *fromC, *fromS;
  int TC, TS, nfc, nfs;
  int4* qnn;
};
LOAM_D MpNnCtx mp_nn_ctx(const MpBuffers& b, int p) {
  MpNnCtx c;
  c.stack = b.stack + (size_t)p * b.cap_stack;
  c.hcs = b.hC_start + (size_t)p * (b.tmax + 1);
  c.hss = b.hS_start + (size_t)p * (b.tmax + 1);
  c.hcr = b.hC_rec + (size_t)p * b.tmax;
  c.hsr = b.hS_rec + (size_t)p * b.tmax;
  c.hcp = b.hC_pts + (size_t)p * b.map_cap;
  c.hsp = b.hS_pts + (size_t)p * b.map_cap;
  c.TC = b.hC_T[p];
  c.TS = b.hS_T[p];
  c.nfc = b.nfrom[p * 2 + 0];
  c.nfs = b.nfrom[p * 2 + 1];
  c.fromC = b.from + (size_t)p * b.map_cap;
  c.fromS = c.fromC + c.nfc;
  c.qnn = b.q_nn + (size_t)p * b.cap_stack * 2;
  return c;
}

// the list's start: five copies of the seed bound B (see mp_nn_query), or sentinels; n0 / n1: the
// previous iteration's ordered 5-NN (i0..i3 | i4, -, distinct) when !first
LOAM_D void mp_nn_seed_from(const MpNnCtx& c, int q, bool corner, bool first, int4 n0, int4 n1, float4 sel, Top5& t,
                            int& work) {
  float bd = 3.4e38f;
  int bi = 0x7fffffff;
  if (!first) {
    // The previous iteration's five neighbours (when they were five distinct points, n1.z) bound the
    // search: B = the largest of their (distance, index) keys at the moved query.  The list starts
    // as five copies of B and takes only keys below B, so it ends with the points below B — the
    // true 5-NN whenever they lie in the searched cells, the B point itself filling the fifth place
    // when only four lie below it (B is a real point) — and no seed needs to be offered or
    // recognised when the walk meets it again
    if (n1.z) {
      const int prev[5] = {n0.x, n0.y, n0.z, n0.w, n1.x};
      const float4* from = corner ? c.fromC : c.fromS;
      uint64_t B = 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        LOAM_CHECK(prev[k] >= 0 && prev[k] < (corner ? c.nfc : c.nfs), prev[k], q);
        const float4 a = from[prev[k]];
        const uint64_t key = top5_key(sqdist(a.x, a.y, a.z, sel.x, sel.y, sel.z), prev[k]);
        B = key > B ? key : B;
      }
      work += 5;
      bd = __uint_as_float((uint32_t)(B >> 32));
      bi = (int)(uint32_t)B;
    }
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) { t.d[k] = bd; t.i[k] = bi; }
}

LOAM_D void mp_nn_seed(const MpNnCtx& c, int q, bool corner, bool first, float4 sel, Top5& t, int& work) {
  int4 n0 = make_int4(0, 0, 0, 0), n1 = n0;
  if (!first) { n0 = c.qnn[2 * q]; n1 = c.qnn[2 * q + 1]; }
  mp_nn_seed_from(c, q, corner, first, n0, n1, sel, t, work);
}

// the seeds for the next iteration only when the list holds five distinct map points (a rejected
// search can end with copies of B or sentinels; the list is sorted, so copies are adjacent)
LOAM_D int top5_distinct(const Top5& t) {
  return t.i[4] != 0x7fffffff && t.i[0] != t.i[1] && t.i[1] != t.i[2] && t.i[2] != t.i[3] && t.i[3] != t.i[4];
}

LOAM_D void mp_nn_store(const MpNnCtx& c, int q, const Top5& t) {
  c.qnn[2 * q] = make_int4(t.i[0], t.i[1], t.i[2], t.i[3]);
  c.qnn[2 * q + 1] = make_int4(t.i[4], __float_as_int(t.d[4]), top5_distinct(t), 0);
}

template <int S = kMpQueryThreads, int L = 1, int CAPL = 27>
LOAM_D void mp_nn_query(const MpBuffers& b, const MpNnCtx& c, int q, int nsc, bool first, const loampose::MapRot& r,
                        uint32_t* lst, float4& sel, Top5& t, int& work, int sub = 0) {
  const bool corner = q < nsc;
  sel = loampose::point_to_map(r, c.stack[corner ? q : b.capC + (q - nsc)]);
  mp_nn_seed(c, q, corner, first, sel, t, work);
  if (corner) knn5_flat<S, L, CAPL>(c.hcs, c.hcr, c.hcp, c.TC, sel, t, lst, work, sub);
  else knn5_flat<S, L, CAPL>(c.hss, c.hsr, c.hsp, c.TS, sel, t, lst, work, sub);
  if constexpr (L > 1) knn5_merge<L>(t);
  LOAM_CHECK(q < b.cap_stack && (t.i[4] == 0x7fffffff || t.i[4] < (corner ? c.nfc : c.nfs)), q, t.i[4]);
  if (sub == 0) mp_nn_store(c, q, t);
}

// the line (corner: PCA of the 5 neighbours, 3x3 Jacobi, :721-760) or plane (surf: 5x3 QR, :828-850)
// through the ordered 5-NN points nb; jw: this lane's 27 words of LDS scratch for the Jacobi
LOAM_D void mp_fit_compute(bool corner, const float4 (&nb)[5], float* jw, float4& g0, float4& g1) {
  if (corner) {  // :721-760
    float cx = 0, cy = 0, cz = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) { cx += nb[k].x; cy += nb[k].y; cz += nb[k].z; }
    cx /= 5; cy /= 5; cz /= 5;
    float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float ax = nb[k].x - cx, ay = nb[k].y - cy, az = nb[k].z - cz;
      a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
      a22 += ay * ay; a23 += ay * az; a33 += az * az;
    }
    a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
    (void)jw;
    const float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33};
    float D1[3], V1[9];
    loamla::jacobi3_reg(A1, D1, V1);  // (bit-identical to jacobi<3>: tests/test_jacobi3.py)
    const bool valid = D1[0] > 3 * D1[1];
    g0 = make_float4((float)(D(cx) + 0.1 * D(V1[0])), (float)(D(cy) + 0.1 * D(V1[1])),
                     (float)(D(cz) + 0.1 * D(V1[2])), valid ? 1.0f : 0.0f);
    g1 = make_float4((float)(D(cx) - 0.1 * D(V1[0])), (float)(D(cy) - 0.1 * D(V1[1])),
                     (float)(D(cz) - 0.1 * D(V1[2])), 0.0f);
  } else {  // :828-850
    float A0[15], B0[5] = {-1, -1, -1, -1, -1}, X0[3], ws[14];
#pragma unroll
    for (int k = 0; k < 5; ++k) { A0[k * 3 + 0] = nb[k].x; A0[k * 3 + 1] = nb[k].y; A0[k * 3 + 2] = nb[k].z; }
    loamla::qr_solve(A0, B0, 5, 3, X0, ws);
    float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
    const float ps = (float)sqrt(D(pa * pa + pb * pb + pc * pc));
    pa /= ps; pb /= ps; pc /= ps; pd /= ps;
    bool planeValid = true;
#pragma unroll
    for (int k = 0; k < 5; ++k)
      if (fabs(D(pa * nb[k].x + pb * nb[k].y + pc * nb[k].z + pd)) > 0.2) planeValid = false;
    g0 = make_float4(pa, pb, pc, pd);
    g1 = make_float4(planeValid ? 1.0f : 0.0f, 0.0f, 0.0f, 0.0f);
  }
}

// the weighted residual of the mapped point sel against a fit (:762-816 corner, :852-874 surf)
LOAM_D void mp_fit_residual(bool corner, float4 g0, float4 g1, float4 sel, float4& cf, int& ok) {
  ok = 0;
  cf = make_float4(0, 0, 0, 0);
  if (corner && g0.w != 0.0f) {  // :762-816
    const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
    const float x1 = g0.x, y1 = g0.y, z1 = g0.z, x2 = g1.x, y2 = g1.y, z2 = g1.z;
    const float m11 = (x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1);
    const float m22 = (x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1);
    const float m33 = (y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1);
    const float a012 = (float)sqrt(D(m11 * m11 + m22 * m22 + m33 * m33));
    const float l12 = (float)sqrt(D((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2)));
    const float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
    const float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
    const float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
    const float ld2 = a012 / l12;
    const float sw = (float)(1 - 0.9 * fabs(D(ld2)));
    cf = make_float4(sw * la, sw * lb, sw * lc, sw * ld2);
    ok = D(sw) > 0.1 ? 1 : 0;
  } else if (!corner && g1.x != 0.0f) {  // :852-874
    const float pa = g0.x, pb = g0.y, pc = g0.z, pd = g0.w;
    const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
    const float sw = (float)(1 - 0.9 * fabs(D(pd2)) / sqrt(sqrt(D(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z))));
    cf = make_float4(sw * pa, sw * pb, sw * pc, sw * pd2);
    ok = D(sw) > 0.1 ? 1 : 0;
  }
}

// jw: this lane's 27 words of LDS scratch for the 3x3 Jacobi
LOAM_D void mp_fit_query(const MpBuffers& b, int p, int q, int nsc, bool first, int4 n0, int4 n1, float4 sel,
                         float* jw, int& nfits, float4& cf, int& ok) {
  const bool corner = q < nsc;
  const int nfc = b.nfrom[p * 2 + 0];
  const float4* from = b.from + (size_t)p * b.map_cap + (corner ? 0 : nfc);
  MpFit* qfit = (MpFit*)b.q_fit + (size_t)p * b.cap_stack;
  ok = 0;
  cf = make_float4(0, 0, 0, 0);
  if (n1.x != 0x7fffffff && D(__int_as_float(n1.y)) < 1.0) {  // :719, :826
    MpFit f = qfit[q];
    if (first || f.n0.x != n0.x || f.n0.y != n0.y || f.n0.z != n0.z || f.n0.w != n0.w || f.n1.x != n1.x) {
      ++nfits;
      const int idx[5] = {n0.x, n0.y, n0.z, n0.w, n1.x};
      float4 nb[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        LOAM_CHECK(idx[k] >= 0 && idx[k] < (corner ? nfc : b.nfrom[p * 2 + 1]), idx[k], q);
        nb[k] = from[idx[k]];
      }
      f.n0 = n0;
      f.n1 = make_int4(n1.x, 0, 0, 0);
      mp_fit_compute(corner, nb, jw, f.g0, f.g1);
      qfit[q] = f;
    }
    mp_fit_residual(corner, f.g0, f.g1, sel, cf, ok);
  } else if (first) {
    // no fit this iteration: drop a fit left by an earlier frame (whose map indices name other
    // points) so that a later iteration cannot take it for this frame's
    qfit[q].n0 = make_int4(-1, -1, -1, -1);
  }
}

// sin / cos of the TobeMapped rotation for the rows
struct MpTrig {
  float srx, crx, sry, cry, srz, crz;
};
LOAM_D MpTrig mp_trig_of(const float* trig) { return {trig[0], trig[1], trig[2], trig[3], trig[4], trig[5]}; }
// the same values from the stored rotation (rot_store: dsin / dcos of the same TobeMapped angles),
// without the serial double sin / cos in the kernel prologue
LOAM_D MpTrig mp_trig_of(const loampose::MapRot& r) {
  return {(float)r.s0, (float)r.c0, (float)r.s1, (float)r.c1, (float)r.s2, (float)r.c2};
}

// the accepted row's J (:897-921): a[0..5] and b = -coefficient.w
LOAM_D void mp_row_jac(const MpTrig& tg, float4 o, float4 c, float (&a)[6], float& bb) {
  const float srx = tg.srx, crx = tg.crx, sry = tg.sry, cry = tg.cry, srz = tg.srz, crz = tg.crz;
  a[0] = (crx * sry * srz * o.x + crx * crz * sry * o.y - srx * sry * o.z) * c.x +
         (-srx * srz * o.x - crz * srx * o.y - crx * o.z) * c.y +
         (crx * cry * srz * o.x + crx * cry * crz * o.y - cry * srx * o.z) * c.z;
  a[1] = ((cry * srx * srz - crz * sry) * o.x + (sry * srz + cry * crz * srx) * o.y + crx * cry * o.z) * c.x +
         ((-cry * crz - srx * sry * srz) * o.x + (cry * srz - crz * srx * sry) * o.y - crx * sry * o.z) * c.z;
  a[2] = ((crz * srx * sry - cry * srz) * o.x + (-cry * crz - srx * sry * srz) * o.y) * c.x +
         (crx * crz * o.x - crx * srz * o.y) * c.y +
         ((sry * srz + cry * crz * srx) * o.x + (crz * sry - cry * srx * srz) * o.y) * c.z;
  a[3] = c.x;
  a[4] = c.y;
  a[5] = c.z;
  bb = -c.w;
}

LOAM_D void mp_row_accum(const MpTrig& tg, float4 o, float4 c, double (&acc)[28]) {
  float a[6], bb;
  mp_row_jac(tg, o, c, a, bb);
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int jj = i; jj < 6; ++jj) { acc[k] = loamla::dmac(acc[k], a[i], a[jj]); ++k; }
#pragma unroll
  for (int i = 0; i < 6; ++i) acc[21 + i] = loamla::dmac(acc[21 + i], a[i], bb);
  acc[27] += 1.0;
}

struct MpStepScratch {
  float lm_ws[loamla::kLmWs];
  int lm_iws[12];
  float AtA[36], AtB[6], X[6];
  float jE[6], jV[36];  // iteration 0: jacobi6_wave's eigen decomposition of AtA
};

// the first wave of the workgroup (the iteration-0 eigen decomposition, jacobi6_wave), the rest on
// lane 0: iteration bookkeeping, the 6x6 step when there are >= 50 rows (:886-889), the update (no
// NaN guard in mapping, :956-961) and the convergence test (:972)
LOAM_D void mp_step(const MpBuffers& b, int p, const double* tot, MpStepScratch& sh) {
  const int lane = lane_id();
  int* ist = b.istate + (size_t)p * kMpStateInts;
  float* st = b.state + (size_t)p * kMpStateFloats;
  const int iter = ist[kMiIters];
  const int nrows = (int)tot[27];
  // lane 0's global reads of the step, issued together up front (round trips on the serial chain)
  int c_rows = 0, degen = 0, c_deg = 0;
  float T[6] = {0, 0, 0, 0, 0, 0};
  if (lane == 0) {
    c_rows = ist[kMiRows];
    degen = ist[kMiDegen];
    c_deg = ist[kMiDegSteps];
#pragma unroll
    for (int q = 0; q < 6; ++q) T[q] = st[kMpTobe + q];
  }
  if (nrows >= 50 && lane == 0) {
    int k = 0;
    for (int i = 0; i < 6; ++i)
      for (int jj = i; jj < 6; ++jj) {
        sh.AtA[i * 6 + jj] = (float)tot[k];
        sh.AtA[jj * 6 + i] = (float)tot[k];
        ++k;
      }
    for (int i = 0; i < 6; ++i) sh.AtB[i] = (float)tot[21 + i];
  }
  const bool solve = nrows >= 50;  // (uniform)
  bool eig = solve && iter == 0, cert = false;
  if (solve) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();  // lane 0's AtA / AtB, for the wave
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (eig) {
      cert = loamla::nondegenerate_certified(sh.AtA, 100.0f);  // every lane, the same answer
      eig = !cert;
      if (eig) loamla::jacobi6_wave(sh.AtA, sh.jE, sh.jV);
    }
    // the QR solve by the whole wave; lane 0 goes on with X
    loamla::lm_step_wave(sh.AtA, sh.AtB, iter, 100.0f, &degen, st + kMpMatP, sh.X, sh.lm_ws, sh.lm_iws,
                         eig ? sh.jE : nullptr, eig ? sh.jV : nullptr, cert);
  }
  if (lane != 0) return;
  ist[kMiIters] = iter + 1;
  ist[kMiRows] = c_rows + nrows;
  if (solve) {
    ist[kMiDegen] = degen;
    if (degen) ist[kMiDegSteps] = c_deg + 1;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      T[q] = T[q] + sh.X[q];
      st[kMpTobe + q] = T[q];
    }
    rot_store(b, p, T);
    const float dR = loamla::delta_r(sh.X), dT = loamla::delta_t(sh.X);
    if (D(dR) < 0.05 && D(dT) < 0.05) ist[kMiStop] = 1;
  }
  if (iter + 1 >= b.max_iter) ist[kMiStop] = 1;
}
}  // namespace

// the fused step of one-wave workgroups (k_mp_nnfit<true>): the wave's row sums as
// this workgroup's partial (write-through), and the last workgroup of the instance to arrive sums
// the G partials in workgroup order and runs the step
// red: the wave's sums reduce-scattered (wave_reduce_scatter_28: lanes 2v, 2v+1 hold value v)
LOAM_D void mp_store_partial_and_step(const MpBuffers& b, int p, int wg, int G, double red) {
  static_assert(kMpFitThreads == 64, "one wave per workgroup: the wave's sums are the partial");
  const int lane = lane_id();
  if ((lane & 1) == 0 && (lane >> 1) < 28)
    store_partial(&b.part[((size_t)p * kMpFitGridMax + wg) * 28 + (lane >> 1)], red);
  __shared__ int sh_last;
  __shared__ double tot[28];
  __shared__ MpStepScratch sh;
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) sh_last = arrive_last(&b.done[p], G);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (!sh_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  {  // fixed order over the workgroups: lane (half h, value v) sums half h of the partials in
     // order, sixteen loads in flight per round, then the two halves are added in order
    const int v = lane % 28, h = lane / 28, G2 = (G + 1) / 2;
    const int g0 = h == 0 ? 0 : G2, g1 = h == 0 ? G2 : G;
    const double* pp = b.part + (size_t)p * kMpFitGridMax * 28 + v;
    double sum = 0.0;
    if (h < 2) {
      for (int g = g0; g < g1; g += 16) {
        double t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          t[u] = g + u < g1 ? __hip_atomic_load(&pp[(size_t)(g + u) * 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (g + u < g1) sum += t[u];
      }
    }
    const double upper = __shfl_down(sum, 28, 64);
    if (lane < 28) tot[lane] = sum + upper;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (lane == 0) b.done[p] = 0;
  mp_step(b, p, tot, sh);
}
// One mapping L-M iteration's correspondences in one launch: lane per query, the 5-NN search
// (knn5_flat, seeded) then the fit and row — the fit needs only the lane's own five neighbours —
// in one-wave workgroups whose 27-entry candidate lists and 27-word Jacobi scratch share one LDS
// array (the wave's search is over before its fits begin).  Rows in query order per workgroup.
// FUSED: the workgroup's partial + the last workgroup's step (mp_store_partial_and_step); else the
// rows go to q_ok / q_cf for k_mp_iter.  COUNT: the work counters.
#ifndef LOAM_NNFIT_WPE
#define LOAM_NNFIT_WPE 4
#endif
template <bool FUSED, bool COUNT>
__global__ __launch_bounds__(kMpFitThreads) __attribute__((amdgpu_waves_per_eu(LOAM_NNFIT_WPE))) void k_mp_nnfit(MpBuffers b) {
  constexpr int NT = kMpFitThreads;
  static_assert(NT == 64, "the list / scratch sharing needs one wave per workgroup");
  const XcdBlock blk = xcd_block();
  const int p = blk.y, tid = threadIdx.x;
  int* ist = b.istate + (size_t)p * kMpStateInts;
  if (!ist[kMiLmRan] || ist[kMiStop]) return;
  const bool first = ist[kMiIters] == 0;
  __shared__ uint32_t lds[kNnListCap * NT];  // candidate lists (column tid, stride NT) / Jacobi rows
  const int nsc = b.sseg_cnt[p * 2 + 0], nss = b.sseg_cnt[p * 2 + 1];
  const int nq = nsc + nss;
  int8_t* qok = b.q_ok + (size_t)p * b.cap_stack;
  float4* qcf = b.q_cf + (size_t)p * b.cap_stack;
  const loampose::MapRot r = rot_load(b, p);
  const MpNnCtx c = mp_nn_ctx(b, p);
  const MpTrig tg = mp_trig_of(r);
  float* jw = (float*)lds + tid * 27;
  int nfits = 0, work = 0;
  // FUSED: the rows of each pass over the queries are reduce-scattered over the wave at once (no
  // 28 fp64 sums live across the search), the passes' sums added in pass order (one pass per lane
  // for a VLP-16 stack)
  double red = 0.0;
  // FUSED: lane 2t's term t of the 28 sums (JᵀJ upper triangle row-major, Jᵀb, rows) as the
  // product of row entries term_x * term_y (mp_row_accum's order; entry 7 = 1 per accepted row)
  int term_x = -1, term_y = -1;
  if (FUSED && (tid & 1) == 0 && (tid >> 1) < 28) {
    const int t = tid >> 1;
    if (t < 21) {
      int i = 0, r0 = t;
      while (r0 >= 6 - i) { r0 -= 6 - i; ++i; }
      term_x = i;
      term_y = i + r0;
    } else if (t < 27) {
      term_x = t - 21;
      term_y = 6;
    } else {
      term_x = 7;
      term_y = 7;
    }
  }
  // one record per query (MpFit in q_fit): the 5-NN of the last iteration (i0..i3 | i4, 0,
  // distinct, fit valid) and the fit made for them — the seeds and the reuse test in one read
  MpFit* qrec = (MpFit*)b.q_fit + (size_t)p * b.cap_stack;
  for (int q0 = blk.x * NT; q0 < nq; q0 += gridDim.x * NT) {  // (wave-uniform trip count)
    const int q = q0 + tid;
    const bool corner = q < nsc;
    float4 sel = make_float4(0, 0, 0, 0), o = sel, cf = sel;
    int4 r0 = make_int4(-1, -1, -1, -1), r1 = make_int4(0, 0, 0, 0);
    bool row_ok = false;
    Top5 t;
    if (q < nq) {
      o = c.stack[corner ? q : b.capC + (q - nsc)];
      if (!first) { r0 = qrec[q].n0; r1 = qrec[q].n1; }
      sel = loampose::point_to_map(r, o);
      mp_nn_seed_from(c, q, corner, first, r0, r1, sel, t, work);
      if (corner) knn5_flat<NT, 1, kNnListCap>(c.hcs, c.hcr, c.hcp, c.TC, sel, t, lds + tid, work, 0);
      else knn5_flat<NT, 1, kNnListCap>(c.hss, c.hsr, c.hsp, c.TS, sel, t, lds + tid, work, 0);
#ifdef LOAM_DIAG_SEARCH2  // (diagnostic build: the search twice, its cost measured by the difference)
      {
        Top5 t2;
        int w2 = 0;
        asm volatile("" ::: "memory");
        mp_nn_seed_from(c, q, corner, first, r0, r1, sel, t2, w2);
        if (corner) knn5_flat<NT, 1, kNnListCap>(c.hcs, c.hcr, c.hcp, c.TC, sel, t2, lds + tid, w2, 0);
        else knn5_flat<NT, 1, kNnListCap>(c.hss, c.hsr, c.hsp, c.TS, sel, t2, lds + tid, w2, 0);
        if (t2.i[0] != t.i[0]) nfits += 1 << 20;
      }
#endif
      LOAM_CHECK(q < b.cap_stack && (t.i[4] == 0x7fffffff || t.i[4] < (corner ? c.nfc : c.nfs)), q, t.i[4]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();  // every lane's list reads are done before the scratch reuse
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (q < nq) {
      const int4 n0 = make_int4(t.i[0], t.i[1], t.i[2], t.i[3]);
      // the stored fit is this list's when the list is unchanged and the fit was made (a fit is
      // a function of the five map points alone: reusing it is bit-identical to refitting)
      bool valid = !first && r1.w && r0.x == n0.x && r0.y == n0.y && r0.z == n0.z && r0.w == n0.w &&
                   r1.x == t.i[4];
      int ok = 0;
      if (t.i[4] != 0x7fffffff && D(t.d[4]) < 1.0) {  // :719, :826
        float4 g0, g1;
        if (valid) {
          g0 = qrec[q].g0;
          g1 = qrec[q].g1;
        } else {
          ++nfits;
          const float4* from = corner ? c.fromC : c.fromS;
          float4 nb[5];
#pragma unroll
          for (int k = 0; k < 5; ++k) {
            LOAM_CHECK(t.i[k] >= 0 && t.i[k] < (corner ? c.nfc : c.nfs), t.i[k], q);
            nb[k] = from[t.i[k]];
          }
          mp_fit_compute(corner, nb, jw, g0, g1);
#ifdef LOAM_DIAG_FIT2  // (diagnostic build: every fit twice)
          {
            float4 h0, h1;
            asm volatile("" ::: "memory");
            mp_fit_compute(corner, nb, jw, h0, h1);
            if (h0.x != g0.x) nfits += 1 << 20;
          }
#endif
          qrec[q].g0 = g0;
          qrec[q].g1 = g1;
          valid = true;
        }
        mp_fit_residual(corner, g0, g1, sel, cf, ok);
      }
      // the record is written only when it changes: a reused fit's list is the stored one (the
      // next iteration's seeds and reuse test read indices and flags only)
      const int4 n1 = make_int4(t.i[4], 0, top5_distinct(t), valid ? 1 : 0);
      if (first || r0.x != n0.x || r0.y != n0.y || r0.z != n0.z || r0.w != n0.w || r1.x != n1.x || r1.z != n1.z ||
          r1.w != n1.w) {
        qrec[q].n0 = n0;
        qrec[q].n1 = n1;
      }
      if constexpr (!FUSED) {  // (k_mp_iter reads the rows back; the fused step sums them below)
        qok[q] = (int8_t)ok;
        qcf[q] = cf;
      }
      row_ok = ok != 0;
    }
    if constexpr (FUSED) {  // (outside the branch: every lane takes part)
      // the pass's rows through LDS (8 floats per lane: J, b, 1 when accepted, else zeros), then
      // lane 2t sums term t over the wave's rows in query order: no 28 fp64 sums per lane
      float a6[6] = {0, 0, 0, 0, 0, 0}, bb = 0.0f;
      if (row_ok) mp_row_jac(tg, o, cf, a6, bb);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();  // the fits' scratch reads are done
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      float* rw = (float*)lds + tid * 8;
#pragma unroll
      for (int k = 0; k < 6; ++k) rw[k] = a6[k];
      rw[6] = bb;
      rw[7] = row_ok ? 1.0f : 0.0f;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (term_x >= 0) {
        const float* rows = (const float*)lds;
        double s = 0.0;
#pragma unroll 16
        for (int l = 0; l < NT; ++l) s = loamla::dmac(s, rows[l * 8 + term_x], rows[l * 8 + term_y]);
        red += s;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();  // the fits' scratch is free before the next lists
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  nfits = wave_sum(nfits);
  if (lane_id() == 0 && nfits) atomicAdd(&ist[kMiFits], nfits);
  if (COUNT) {
    const int ncand = wave_sum(work & ((1 << kWorkCellShift) - 1)), ncell = wave_sum(work >> kWorkCellShift);
    if (lane_id() == 0 && ncand) {
      atomicAdd(&ist[kMiNnCand], ncand);
      atomicAdd(&ist[kMiNnCells], ncell);
    }
  }
  if constexpr (FUSED) mp_store_partial_and_step(b, p, blk.x, (int)gridDim.x, red);
}

namespace {
struct MpIterShared {
  double red[16][28];  // (up to 1024 threads)
  double tot[28];
  float trig[6];
  MpStepScratch step;
};
}  // namespace

// the normal equations of the accepted rows (:879-974) and the 6x6 step, one workgroup per
// instance; rows = the accepted correspondences of this iteration, in stack order
// NT threads per instance: 256 for large batches, 1024 for small ones (a shorter row chain per lane)
template <int NT>
__global__ __launch_bounds__(NT) void k_mp_iter(MpBuffers b) {
  const int p = blockIdx.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  int* ist = b.istate + (size_t)p * kMpStateInts;
  if (!ist[kMiLmRan] || ist[kMiStop]) return;
  __shared__ MpIterShared sh;
  const int nsc = b.sseg_cnt[p * 2 + 0], nss = b.sseg_cnt[p * 2 + 1];
  const int nq = nsc + nss;
  const float4* stack = b.stack + (size_t)p * b.cap_stack;
  const int8_t* qok = b.q_ok + (size_t)p * b.cap_stack;
  const float4* qcf = b.q_cf + (size_t)p * b.cap_stack;
  const MpTrig tg = mp_trig_of(rot_load(b, p));
  const float srx = tg.srx, crx = tg.crx, sry = tg.sry, cry = tg.cry, srz = tg.srz, crz = tg.crz;
  double acc[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) acc[k] = 0.0;
  // four rows' loads in flight per step; the rows are still summed in the lane's q order
  for (int q0 = tid; q0 < nq; q0 += 4 * NT) {  // :897-921
    int8_t okv[4];
    float4 ov[4], cv4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = q0 + u * NT;
      okv[u] = q < nq ? qok[q] : (int8_t)0;
      ov[u] = q < nq ? stack[q < nsc ? q : b.capC + (q - nsc)] : make_float4(0, 0, 0, 0);
      cv4[u] = q < nq ? qcf[q] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    if (!okv[u]) continue;
    const float4 o = ov[u], c = cv4[u];
    float a[6];
    a[0] = (crx * sry * srz * o.x + crx * crz * sry * o.y - srx * sry * o.z) * c.x +
           (-srx * srz * o.x - crz * srx * o.y - crx * o.z) * c.y +
           (crx * cry * srz * o.x + crx * cry * crz * o.y - cry * srx * o.z) * c.z;
    a[1] = ((cry * srx * srz - crz * sry) * o.x + (sry * srz + cry * crz * srx) * o.y + crx * cry * o.z) * c.x +
           ((-cry * crz - srx * sry * srz) * o.x + (cry * srz - crz * srx * sry) * o.y - crx * sry * o.z) * c.z;
    a[2] = ((crz * srx * sry - cry * srz) * o.x + (-cry * crz - srx * sry * srz) * o.y) * c.x +
           (crx * crz * o.x - crx * srz * o.y) * c.y +
           ((sry * srz + cry * crz * srx) * o.x + (crz * sry - cry * srx * srz) * o.y) * c.z;
    a[3] = c.x;
    a[4] = c.y;
    a[5] = c.z;
    const float bb = -c.w;
    int k = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int jj = i; jj < 6; ++jj) acc[k++] += (double)a[i] * (double)a[jj];  // (dmac measured slower here)
#pragma unroll
    for (int i = 0; i < 6; ++i) acc[21 + i] += (double)a[i] * (double)bb;
    acc[27] += 1.0;
  }
  }
  wave_reduce_scatter_28(acc);  // lanes 2v, 2v+1: the wave sum of value v
  if ((lane & 1) == 0 && (lane >> 1) < 28) sh.red[w][lane >> 1] = acc[0];
  __syncthreads();
  if (tid < 28) {
    double v = sh.red[0][tid];
    for (int ww = 1; ww < NT / 64; ++ww) v += sh.red[ww][tid];
    sh.tot[tid] = v;
  }
  __syncthreads();
  if (tid < 64) mp_step(b, p, sh.tot, sh.step);  // the first wave
}


// Small batches (streaming, config 2): the whole iteration in one launch — each lane its query's
// 5-NN, fit and row, fp64 partials per workgroup, and the last workgroup of the instance to finish
// sums them in a fixed order and runs the step (three launches and a one-workgroup row pass fewer
// per iteration).
__global__ __launch_bounds__(kMpQueryThreads) void k_mp_lm_small(MpBuffers b) {
  const int p = blockIdx.y, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  int* ist = b.istate + (size_t)p * kMpStateInts;
  if (!ist[kMiLmRan] || ist[kMiStop]) return;
  LOAM_PH(const unsigned long long ph0 = ph_now(); if (tid == 0) ph_start(&g_ph_mp, ph0);)
  __shared__ uint32_t lists[27 * kMpQueryThreads];
  __shared__ float jac[kMpQueryThreads][27];
  __shared__ double red[kMpQueryThreads / 64][28];
  const int nsc = b.sseg_cnt[p * 2 + 0], nss = b.sseg_cnt[p * 2 + 1];
  const int nq = nsc + nss;
  const float4* stack = b.stack + (size_t)p * b.cap_stack;
  int8_t* qok = b.q_ok + (size_t)p * b.cap_stack;
  float4* qcf = b.q_cf + (size_t)p * b.cap_stack;
  const bool first = ist[kMiIters] == 0;
  const loampose::MapRot r = rot_load(b, p);
  const MpNnCtx c = mp_nn_ctx(b, p);
  int work = 0, nfits = 0;  // (work: the batch kernel's profiling counter; not summed here)
  const MpTrig tg = mp_trig_of(r);
  double acc[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) acc[k] = 0.0;
  // each lane's row is added right after its fit (same queries, same order per lane as a
  // separate pass over the stored rows: identical sums, one reload round trip fewer)
  // kMpNnLanes lanes per query: the 5-NN search split over the group, the fit and row on its first lane
  constexpr int L = kMpNnLanes, QPB = kMpQueryThreads / L;
  const int sub = tid % L;
  for (int q = blockIdx.x * QPB + tid / L; q < nq; q += gridDim.x * QPB) {
    LOAM_PH(const unsigned long long pq0 = ph_now();)
    float4 sel;
    Top5 t;
    mp_nn_query<kMpQueryThreads, L>(b, c, q, nsc, first, r, lists + tid, sel, t, work, sub);
    LOAM_PH(asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); const unsigned long long pq1 = ph_now();)
    float4 cf = make_float4(0, 0, 0, 0);
    int ok = 0;
    if (sub == 0) {
      mp_fit_query(b, p, q, nsc, first, make_int4(t.i[0], t.i[1], t.i[2], t.i[3]),
                   make_int4(t.i[4], __float_as_int(t.d[4]), 0, 0), sel, jac[tid], nfits, cf, ok);
      qok[q] = (int8_t)ok;
      qcf[q] = cf;
      if (ok) mp_row_accum(tg, stack[q < nsc ? q : b.capC + (q - nsc)], cf, acc);
    }
    LOAM_PH(asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); const unsigned long long pq2 = ph_now();
            if (lane == 0) ph_query(&g_ph_mp, first ? 0 : 1, pq1 - pq0, pq2 - pq1);)
  }
  nfits = wave_sum(nfits);
  if (lane == 0 && nfits) atomicAdd(&ist[kMiFits], nfits);
  wave_reduce_scatter_28(acc);
  if ((lane & 1) == 0 && (lane >> 1) < 28) red[w][lane >> 1] = acc[0];
  __syncthreads();
  const int G = (int)gridDim.x;
  if (tid < 28) {
    double v = red[0][tid];
    for (int ww = 1; ww < kMpQueryThreads / 64; ++ww) v += red[ww][tid];
    store_partial(&b.part[((size_t)p * kMpSmallGrid + blockIdx.x) * 28 + tid], v);
  }
  __shared__ int sh_last;
  __shared__ double slice[8][28];
  __shared__ double tot[28];
  __shared__ MpStepScratch sh;
  __syncthreads();
  LOAM_PH(const int phk = first ? 0 : 1; const unsigned long long ph1 = ph_now();
          if (tid == 0) ph_arrive(&g_ph_mp, phk, ph0, ph1);)
  // (store_partial / arrive_last: the partials are drained write-through before the counter add;
  // the last workgroup acquires at agent scope, then reads them with sc1 loads)
  if (tid == 0)
    sh_last = arrive_last(&b.done[p], G);
  __syncthreads();
  if (!sh_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  LOAM_PH(const unsigned long long ph2 = ph_now();)
  if (tid < 8 * 28) {  // fixed-order sum: slice s holds partials s, s + 8, ... (all in flight)
    const int v = tid % 28, sl = tid / 28;
    const double* pp = b.part + (size_t)p * kMpSmallGrid * 28 + v;
    double t8[kMpSmallGrid / 8];
#pragma unroll
    for (int u = 0; u < kMpSmallGrid / 8; ++u) {
      const int g = sl + 8 * u;
      t8[u] = g < G ? __hip_atomic_load(&pp[(size_t)g * 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    }
    double a1 = 0.0;
#pragma unroll
    for (int u = 0; u < kMpSmallGrid / 8; ++u)
      if (sl + 8 * u < G) a1 += t8[u];
    slice[sl][v] = a1;
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
    mp_step(b, p, tot, sh);
    LOAM_PH(const unsigned long long ph4 = ph_now(); if (tid == 0) ph_last(&g_ph_mp, phk, ph1, ph2, ph3, ph4);)
  }
}

// ---- the one-instance mapping L-M as one persistent launch (streaming: config 3, config 2) ----
// k_mp_lm_small's iteration (5-NN, fit, row per query group of kMpNnLanes lanes) for every
// iteration in one launch, as k_od_lm_stream does for the odometry: a query stays on the same
// lanes for the whole loop (its 5-NN seeds and fit record are read back by the lanes that wrote
// them), the partial sums are exchanged per iteration with write-through stores and a publication
// word per workgroup, and every workgroup sums all G partials in workgroup order and runs the step
// on its own copy of the state: the same transform and the same convergence decision everywhere.
struct MpLsState {
  float T[6], matP[36];
  int degen, iters, rows, deg_steps, stop;
};

// mp_step on the workgroup-local state (the first wave): the same arithmetic and decisions
LOAM_D void mp_step_ls(int max_iter, const double* tot, MpLsState& S, MpStepScratch& sh) {
  const int lane = lane_id();
  const int iter = S.iters;
  const int nrows = (int)tot[27];
  if (nrows >= 50 && lane == 0) {
    int k = 0;
    for (int i = 0; i < 6; ++i)
      for (int jj = i; jj < 6; ++jj) {
        sh.AtA[i * 6 + jj] = (float)tot[k];
        sh.AtA[jj * 6 + i] = (float)tot[k];
        ++k;
      }
    for (int i = 0; i < 6; ++i) sh.AtB[i] = (float)tot[21 + i];
  }
  const bool solve = nrows >= 50;  // (uniform)
  bool eig = solve && iter == 0, cert = false;
  int degen = S.degen;
  if (solve) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (eig) {
      cert = loamla::nondegenerate_certified(sh.AtA, 100.0f);
      eig = !cert;
      if (eig) loamla::jacobi6_wave(sh.AtA, sh.jE, sh.jV);
    }
    loamla::lm_step_wave(sh.AtA, sh.AtB, iter, 100.0f, &degen, S.matP, sh.X, sh.lm_ws, sh.lm_iws,
                         eig ? sh.jE : nullptr, eig ? sh.jV : nullptr, cert);
  }
  if (lane != 0) return;
  S.iters = iter + 1;
  S.rows += nrows;
  if (solve) {
    S.degen = degen;
    if (degen) ++S.deg_steps;
#pragma unroll
    for (int q = 0; q < 6; ++q) S.T[q] = S.T[q] + sh.X[q];
    const float dR = loamla::delta_r(sh.X), dT = loamla::delta_t(sh.X);
    if (D(dR) < 0.05 && D(dT) < 0.05) S.stop = 1;
  }
  if (iter + 1 >= max_iter) S.stop = 1;
}

__global__ __launch_bounds__(kMpQueryThreads) void k_mp_lm_stream(MpBuffers b) {
  const int g = blockIdx.x, G = gridDim.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6, p = 0;
  int* ist = b.istate;
  float* st = b.state;
  if (!ist[kMiLmRan] || ist[kMiStop]) return;  // (the same value in every workgroup)
  __shared__ uint32_t lists[27 * kMpQueryThreads];
  __shared__ float jac[kMpQueryThreads][27];
  __shared__ double red[kMpQueryThreads / 64][28], slice[8][28], tot[28];
  __shared__ MpStepScratch sh;
  __shared__ MpLsState S;
  __shared__ unsigned long long sh_epoch;
  if (tid < 6) S.T[tid] = st[kMpTobe + tid];
  if (tid < 36) S.matP[tid] = st[kMpMatP + tid];
  if (tid == 0) {
    S.degen = ist[kMiDegen];
    S.iters = ist[kMiIters];
    S.rows = ist[kMiRows];
    S.deg_steps = ist[kMiDegSteps];
    S.stop = 0;
    sh_epoch = b.ls_epoch[0];
  }
  __syncthreads();
  const int nsc = b.sseg_cnt[p * 2 + 0], nss = b.sseg_cnt[p * 2 + 1];
  const int nq = nsc + nss;
  const float4* stack = b.stack;
  int8_t* qok = b.q_ok;
  float4* qcf = b.q_cf;
  const MpNnCtx c = mp_nn_ctx(b, p);
  constexpr int L = kMpNnLanes, QPB = kMpQueryThreads / L;
  const int sub = tid % L;
  const unsigned long long tag0 = sh_epoch << 16;  // (iterations + 1 <= 1001 < 2^16: loam_create bounds max_iter)
  int nfits = 0;
  for (int it = 0; it < b.max_iter; ++it) {
    const bool first = S.iters == 0;
    const loampose::MapRot r = loampose::map_rot(S.T);  // (rot_store's values: the same dsin / dcos)
    const MpTrig tg = mp_trig_of(r);
    int work = 0;
    double acc[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) acc[k] = 0.0;
    for (int q = g * QPB + tid / L; q < nq; q += G * QPB) {
      float4 sel;
      Top5 t;
      mp_nn_query<kMpQueryThreads, L>(b, c, q, nsc, first, r, lists + tid, sel, t, work, sub);
      float4 cf = make_float4(0, 0, 0, 0);
      int ok = 0;
      if (sub == 0) {
        mp_fit_query(b, p, q, nsc, first, make_int4(t.i[0], t.i[1], t.i[2], t.i[3]),
                     make_int4(t.i[4], __float_as_int(t.d[4]), 0, 0), sel, jac[tid], nfits, cf, ok);
        qok[q] = (int8_t)ok;
        qcf[q] = cf;
        if (ok) mp_row_accum(tg, stack[q < nsc ? q : b.capC + (q - nsc)], cf, acc);
      }
    }
    wave_reduce_scatter_28(acc);
    if ((lane & 1) == 0 && (lane >> 1) < 28) red[w][lane >> 1] = acc[0];
    __syncthreads();
    const int par = it & 1;
    if (tid < 28) {  // this workgroup's partial, waves in order, stored write-through
      double v = red[0][tid];
      for (int ww = 1; ww < kMpQueryThreads / 64; ++ww) v += red[ww][tid];
      store_partial(&b.ls_part[((size_t)par * kMpSmallGrid + g) * 28 + tid], v);
    }
    if (tid < 64) {
      __builtin_amdgcn_wave_barrier();  // (every lane's store drained: store_partial waits for it)
      if (tid == 0)
        __hip_atomic_store(&b.ls_flag[g], tag0 + (unsigned long long)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < G) {  // every workgroup's partial of this iteration
      const unsigned long long want = tag0 + (unsigned long long)(it + 1);
      while (__hip_atomic_load(&b.ls_flag[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want)
        __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
    if (tid < 8 * 28) {  // fixed order: slice s sums partials s, s + 8, ...; the slices in order
      const int v = tid % 28, sl = tid / 28;
      const double* pp = b.ls_part + (size_t)par * kMpSmallGrid * 28 + v;
      double t8[kMpSmallGrid / 8];
#pragma unroll
      for (int u = 0; u < kMpSmallGrid / 8; ++u) {
        const int gg = sl + 8 * u;
        t8[u] = gg < G ? __hip_atomic_load(&pp[(size_t)gg * 28], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
      }
      double a1 = 0.0;
#pragma unroll
      for (int u = 0; u < kMpSmallGrid / 8; ++u)
        if (sl + 8 * u < G) a1 += t8[u];
      slice[sl][v] = a1;
    }
    __syncthreads();
    if (tid < 28) {
      double v = slice[0][tid];
#pragma unroll
      for (int sl = 1; sl < 8; ++sl) v += slice[sl][tid];
      tot[tid] = v;
    }
    __syncthreads();
    if (tid < 64) mp_step_ls(b.max_iter, tot, S, sh);
    __syncthreads();
    if (S.stop) break;
  }
  nfits = wave_sum(nfits);
  if (lane == 0 && nfits) atomicAdd(&ist[kMiFits], nfits);
  if (g == 0) {  // the state for the kernels after the loop (the same in every workgroup)
    if (tid < 6) st[kMpTobe + tid] = S.T[tid];
    if (tid < 36) st[kMpMatP + tid] = S.matP[tid];
    if (tid == 0) {
      rot_store(b, p, S.T);
      ist[kMiDegen] = S.degen;
      ist[kMiIters] = S.iters;
      ist[kMiRows] = S.rows;
      ist[kMiDegSteps] = S.deg_steps;
      ist[kMiStop] = S.stop;
    }
  }
}

// workgroups of k_mp_lm_stream (kMpSmallGrid, as k_mp_lm_small), or 0 when they could not all be
// resident at once (the per-iteration launches run instead)
int mp_lm_stream_grid() {
  static int cap[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_mp_lm_stream, kMpQueryThreads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      per_cu = cus = 0;
    cap[dev] = std::max(1, per_cu * cus);
  }
  // (a margin of 2: other streams' kernels may hold slots a while; half the grid loops twice)
  return 2 * kMpSmallGrid <= cap[dev] ? kMpSmallGrid : (kMpSmallGrid <= cap[dev] ? kMpSmallGrid / 2 : 0);
}

// transformUpdate (:199-232) for the instances whose L-M ran; the IMU blend (:224-225) when the
// host found IMU data for the odometry stamp
__global__ void k_mp_lm_end(MpBuffers b) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p == 0) { b.vg_cnt[0] = 0; b.vg_cnt[1] = 0; b.vg_cnt[2] = 0; b.vg_cnt[3] = 0; }  // (vg_cubes' lists)
  if (p >= b.P) return;
  const int* ist = b.istate + (size_t)p * kMpStateInts;
  if (!ist[kMiLmRan]) return;
  float* st = b.state + (size_t)p * kMpStateFloats;
  if (ist[kMiImu]) {
    const float imuRollLast = st[kMpImuRP], imuPitchLast = st[kMpImuRP + 1];
    st[kMpTobe + 0] = (float)(0.998 * D(st[kMpTobe + 0]) + 0.002 * D(imuPitchLast));
    st[kMpTobe + 2] = (float)(0.998 * D(st[kMpTobe + 2]) + 0.002 * D(imuRollLast));
    rot_store(b, p, st + kMpTobe);
  }
  for (int k = 0; k < 6; ++k) {
    st[kMpBef + k] = st[kMpSum + k];
    st[kMpAft + k] = st[kMpTobe + k];
  }
}

namespace {

// ---------------------------------------------------------------- insertion (:980-1016)
// one workgroup per instance: cube slot of every stack point (corner, then surf), stable ranks by
// one wave walking the stack in order, per-cube prefix, scatter of the map-frame points.
template <int NT>
__global__ __launch_bounds__(NT) void k_mp_insert(MpBuffers b, int* slot_of, int* rank_of) {
  const int p = blockIdx.x, tid = threadIdx.x, lane = lane_id();
  const int* ist = b.istate + (size_t)p * kMpStateInts;
  const int nsc = b.sseg_cnt[p * 2 + 0], nss = b.sseg_cnt[p * 2 + 1];
  const float4* stack = b.stack + (size_t)p * b.cap_stack;
  const loampose::MapRot r = rot_load(b, p);
  const int cW = ist[kMiCenW], cH = ist[kMiCenH], cD = ist[kMiCenD];
  int* so = slot_of + (size_t)p * b.cap_stack;
  int* ro = rank_of + (size_t)p * b.cap_stack;
  __shared__ int cnt[2][kCubeNum];
  __shared__ int scratch[NT / 64 + 1];
  // the (slot, kind) keys the stack uses, as a bitmap; their dense numbering (prefix popcounts)
  // lets every wave keep its own counts when few keys occur (the usual case: a sweep touches a
  // few dozen cubes)
  constexpr int kKeyWords = (2 * kCubeNum + 31) / 32, kDense = 512, kWaves = NT / 64;
  __shared__ unsigned keybits[kKeyWords];
  __shared__ int keypre[kKeyWords + 1];
  __shared__ int wcnt[kWaves][kDense];
  for (int i = tid; i < 2 * kCubeNum; i += NT) cnt[i / kCubeNum][i % kCubeNum] = 0;
  for (int i = tid; i < kKeyWords; i += NT) keybits[i] = 0u;
  for (int i = tid; i < kWaves * kDense; i += NT) wcnt[i / kDense][i % kDense] = 0;
  __syncthreads();
  const int nst = nsc + nss;
  for (int q = tid; q < nst; q += NT) {
    const float4 a = loampose::point_to_map(r, stack[q < nsc ? q : b.capC + (q - nsc)]);
    const int ci = cube_of(a.x, cW), cj = cube_of(a.y, cH), ck = cube_of(a.z, cD);
    const bool in = ci >= 0 && ci < kCubeW && cj >= 0 && cj < kCubeH && ck >= 0 && ck < kCubeD;
    const int s = in ? cube_index(ci, cj, ck) : -1;
    so[q] = s;
    if (s >= 0) {
      const int key = s * 2 + (q < nsc ? 0 : 1);
      atomicOr(&keybits[key >> 5], 1u << (key & 31));
    }
  }
  __threadfence_block();
  __syncthreads();
  {  // exclusive prefix of the words' popcounts
    constexpr int kPer = (kKeyWords + NT - 1) / NT;
    int sum = 0;
    for (int k = 0; k < kPer; ++k) {
      const int i = tid * kPer + k;
      if (i < kKeyWords) sum += __popc(keybits[i]);
    }
    int tot;
    int run = block_excl_scan<NT>(sum, scratch, tot);
    for (int k = 0; k < kPer; ++k) {
      const int i = tid * kPer + k;
      if (i < kKeyWords) {
        keypre[i] = run;
        run += __popc(keybits[i]);
      }
    }
    if (tid == 0) keypre[kKeyWords] = tot;
  }
  __syncthreads();
  const int nkeys = keypre[kKeyWords];
  if (nkeys <= kDense) {
    // stable ranks, all waves: wave w ranks its contiguous chunk of the stack (in order, per dense
    // key), then each key's chunk counts are prefixed in wave order
    const int w = tid >> 6, chunk = ((nst + kWaves * 64 - 1) / (kWaves * 64)) * 64;
    const int q0 = w * chunk, q1 = min(nst, q0 + chunk);
    constexpr int kAhead = 8;  // slot loads of eight 64-point steps in flight (the walk is load-latency bound)
    int sa[kAhead];
    for (int base = q0; base < q1; base += 64) {
      const int step = ((base - q0) >> 6) % kAhead;
      if (step == 0) {
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
          const int qq = base + u * 64 + lane;
          sa[u] = qq < q1 ? so[qq] : -1;
        }
      }
      const int q = base + lane;
      const bool v = q < q1;
      int s = -1;
#pragma unroll
      for (int u = 0; u < kAhead; ++u)
        if (u == step) s = sa[u];
      const int key = s < 0 ? -1 : s * 2 + (q < nsc ? 0 : 1);
      const int id = key < 0 ? -1 : keypre[key >> 5] + __popc(keybits[key >> 5] & ((1u << (key & 31)) - 1u));
      uint64_t m = __ballot(v && id >= 0);
      int rank = 0;
      while (m) {
        const int leader = __ffsll((unsigned long long)m) - 1;
        const int il = __builtin_amdgcn_readlane(id, leader);
        const uint64_t mm = __ballot(v && id == il);
        const int basecnt = wcnt[w][il];
        if (v && id == il) rank = basecnt + __popcll(mm & lanemask_lt());
        __builtin_amdgcn_wave_barrier();
        if (lane == leader) wcnt[w][il] = basecnt + __popcll(mm);
        __builtin_amdgcn_wave_barrier();
        m &= ~mm;
      }
      if (v) ro[q] = rank;
    }
    __threadfence_block();
    __syncthreads();
    // per dense key: chunk bases in wave order (wcnt becomes the base), total into cnt
    for (int i = tid; i < 2 * kCubeNum; i += NT) {
      if (!(keybits[i >> 5] & (1u << (i & 31)))) continue;
      const int id = keypre[i >> 5] + __popc(keybits[i >> 5] & ((1u << (i & 31)) - 1u));
      int run = 0;
#pragma unroll
      for (int ww = 0; ww < kWaves; ++ww) {
        const int c = wcnt[ww][id];
        wcnt[ww][id] = run;
        run += c;
      }
      cnt[i & 1][i >> 1] = run;
    }
    __threadfence_block();
    __syncthreads();
    for (int q = tid; q < nst; q += NT) {
      const int s = so[q];
      if (s < 0) continue;
      const int key = s * 2 + (q < nsc ? 0 : 1);
      const int id = keypre[key >> 5] + __popc(keybits[key >> 5] & ((1u << (key & 31)) - 1u));
      ro[q] += wcnt[q / chunk][id];
    }
  } else if (tid < 64) {  // many keys: stable ranks by one wave, stack order
    for (int base = 0; base < nsc + nss; base += 64) {
      const int q = base + lane;
      const bool v = q < nsc + nss;
      const int kind = q < nsc ? 0 : 1;
      const int s = v ? so[q] : -1;
      const int key = s < 0 ? -1 : s * 2 + kind;
      uint64_t m = __ballot(v && key >= 0);
      int rank = 0;
      while (m) {
        const int leader = __ffsll((unsigned long long)m) - 1;
        const int kl = __builtin_amdgcn_readlane(key, leader);
        const uint64_t mm = __ballot(v && key == kl);
        const int basecnt = cnt[kl & 1][kl >> 1];
        if (v && key == kl) rank = basecnt + __popcll(mm & lanemask_lt());
        __builtin_amdgcn_wave_barrier();
        if (lane == leader) cnt[kl & 1][kl >> 1] = basecnt + __popcll(mm);
        __builtin_amdgcn_wave_barrier();
        m &= ~mm;
      }
      if (v) ro[q] = rank;
    }
  }
  __syncthreads();
  // exclusive prefix over (kind, cube slot), kind-major: each thread owns a contiguous run of the
  // flattened counts (one block scan instead of one per 256 slots); offsets replace the counts in LDS
  int* ac = b.app_cnt + (size_t)p * kCubeNum * 2;
  int* ao = b.app_off + (size_t)p * kCubeNum * 2;
  {
    constexpr int kFlat = 2 * kCubeNum, kPer = (kFlat + NT - 1) / NT;
    int* cf = &cnt[0][0];
    int sum = 0;
    for (int k = 0; k < kPer; ++k) {
      const int i = tid * kPer + k;
      if (i < kFlat) sum += cf[i];
    }
    int tot;
    int run = block_excl_scan<NT>(sum, scratch, tot);
    for (int k = 0; k < kPer; ++k) {
      const int i = tid * kPer + k;
      if (i < kFlat) {
        const int c = cf[i];
        cf[i] = run;
        run += c;
      }
    }
    __syncthreads();
    for (int i = tid; i < kFlat; i += NT) {
      const int kind = i / kCubeNum, s = i % kCubeNum;
      const int o = cf[i], nx = i + 1 < kFlat ? cf[i + 1] : tot;
      ac[s * 2 + kind] = nx - o;
      ao[s * 2 + kind] = o;
    }
  }
  __threadfence_block();
  __syncthreads();
  float4* app = b.app + (size_t)p * b.cap_stack;
  for (int q = tid; q < nsc + nss; q += NT) {
    const int s = so[q];
    if (s < 0) continue;
    const int kind = q < nsc ? 0 : 1;
    app[ao[s * 2 + kind] + ro[q]] = loampose::point_to_map(r, stack[q < nsc ? q : b.capC + (q - nsc)]);
  }
}

// per valid cube: DS input = old cube content ++ appended points (corner region, then surf region);
// thread per (kind, valid cube) segment, one block scan for the offsets
__global__ __launch_bounds__(kMpThreads) void k_mp_vseg(MpBuffers b) {
  static_assert(2 * kMaxValid <= kMpThreads, "one thread per segment");
  const int p = blockIdx.x, tid = threadIdx.x;
  const int nv = b.istate[(size_t)p * kMpStateInts + kMiNValid];
  const int* slots = slot_table(b, b.pool_cur, p);
  const int* ac = b.app_cnt + (size_t)p * kCubeNum * 2;
  __shared__ int scratch[16];
  const int kind = tid / kMaxValid, v = tid % kMaxValid;
  int n = 0, nold = 0;
  if (tid < 2 * kMaxValid && v < nv) {
    const int ind = b.valid[(size_t)p * kMaxValid + v];
    nold = slots[ind * 4 + 1 + 2 * kind];
    n = nold + ac[ind * 2 + kind];
  }
  int tot;
  const int ex = block_excl_scan<kMpThreads>(n, scratch, tot);
  const int lim = b.map_cap;
  if (tid < 2 * kMaxValid) {
    // the reference order fills segments in (kind, v) order; a segment that would pass the
    // capacity is emptied and flags the instance (as the sequential walk did)
    const bool over = ex + n > lim;
    const int sidx = p * 2 * kMaxValid + tid;
    const int base = (int)((size_t)p * b.map_cap) + (over ? 0 : ex);
    b.vseg_b[sidx] = base;
    b.vseg_e[sidx] = base + (over ? 0 : n);
    b.vseg_leaf[sidx] = kind == 0 ? 0.2f : 0.4f;
    if (over && n > 0) b.istate[(size_t)p * kMpStateInts + kMiErr] |= ERR_CAP_MAP;
    b.vseg_nold[sidx] = nold;
    b.vseg_skip[sidx] = 0;
    if (over || n == 0) {
      b.vseg_cnt[sidx] = 0;  // (not in the VoxelGrid's list)
    } else {
      b.vg_lin[atomicAdd(b.vg_cnt + 2, 1)] = sidx;
      // long segments with a short appended tail: the incremental VoxelGrid may take them
      if (b.tune.vg_merge && n > b.tune.vg_merge_min && nold > 0 && n - nold <= kVgMergeNew)
        b.vg_mlist[atomicAdd(b.vg_cnt + 3, 1)] = sidx;
    }
  }
}

// the DS input of every valid-cube segment, flattened over the instance's points: the segments
// are contiguous in (kind, valid cube) order, so a point finds its segment by binary search over
// their starts (LDS) and copies from the old pool or the appended stack points
__global__ __launch_bounds__(256) void k_mp_vcopy(MpBuffers b) {
  constexpr int NS = 2 * kMaxValid;
  const int p = blockIdx.y, tid = threadIdx.x;
  if (b.istate[(size_t)p * kMpStateInts + kMiErr] & ERR_CAP_MAP) return;
  const int nv = b.istate[(size_t)p * kMpStateInts + kMiNValid];
  const int* slots = slot_table(b, b.pool_cur, p);
  const float4* pool = b.pool + ((size_t)b.pool_cur * b.P + p) * b.map_cap;
  const int* ao = b.app_off + (size_t)p * kCubeNum * 2;
  const float4* app = b.app + (size_t)p * b.cap_stack;
  __shared__ int sb[NS + 1], snold[NS], soff[NS], sapp[NS];
  const int base = (int)((size_t)p * b.map_cap);
  if (tid < NS) {
    const int kind = tid / kMaxValid, v = tid % kMaxValid;
    sb[tid] = b.vseg_b[p * NS + tid] - base;
    int nold = 0, off = 0, ap = 0;
    if (v < nv) {
      const int ind = b.valid[(size_t)p * kMaxValid + v];
      nold = slots[ind * 4 + 1 + 2 * kind];
      off = slots[ind * 4 + 2 * kind];
      ap = ao[ind * 2 + kind];
    }
    snold[tid] = nold;
    soff[tid] = off;
    sapp[tid] = ap;
  }
  if (tid == 0) sb[NS] = b.vseg_e[p * NS + NS - 1] - base;
  __syncthreads();
  const int total = sb[NS];
  for (int i = blockIdx.x * 256 + tid; i < total; i += gridDim.x * 256) {
    int lo = 0, hi = NS - 1;  // last segment whose start is <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sb[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const int t = i - sb[lo];
    b.vin[base + i] = t < snold[lo] ? pool[soff[lo] + t] : app[sapp[lo] + (t - snold[lo])];
  }
}

// new cube store: valid cubes <- their DS output, every other cube <- old ++ appended.  The
// (kind, cube) sizes go to LDS in coalesced passes; each thread then owns a contiguous run of
// them, so the offsets and the non-empty list need one block scan each.
template <int NT>
__global__ __launch_bounds__(NT) void k_mp_compact_table(MpBuffers b) {
  constexpr int N = 2 * kCubeNum, E = (N + NT - 1) / NT;
  const int p = blockIdx.x, tid = threadIdx.x;
  const int nv = b.istate[(size_t)p * kMpStateInts + kMiNValid];
  const int* old = slot_table(b, b.pool_cur, p);
  int* nw = slot_table(b, 1 - b.pool_cur, p);
  const int* ac = b.app_cnt + (size_t)p * kCubeNum * 2;
  __shared__ int16_t vidx[kCubeNum];
  __shared__ int nn[N];
  __shared__ int scratch[NT / 64 + 1];
  for (int s = tid; s < kCubeNum; s += NT) vidx[s] = -1;
  __syncthreads();
  if (tid < nv) vidx[b.valid[(size_t)p * kMaxValid + tid]] = (int16_t)tid;
  __syncthreads();
  int vpts = 0;
  for (int x = tid; x < N; x += NT) {
    const int kind = x / kCubeNum, s = x % kCubeNum, v = vidx[s];
    const int n = v >= 0 ? b.vseg_cnt[p * 2 * kMaxValid + kind * kMaxValid + v] : old[s * 4 + 1 + 2 * kind] + ac[s * 2 + kind];
    nn[x] = n;
    if (v >= 0) vpts += n;
  }
  __syncthreads();
  const int x0 = tid * E, x1 = min(N, x0 + E);
  int sum = 0;
  for (int x = x0; x < x1; ++x) sum += nn[x];
  int run;
  int off = block_excl_scan<NT>(sum, scratch, run);
  for (int x = x0; x < x1; ++x) {  // counts -> offsets, in LDS
    const int c = nn[x];
    nn[x] = off;
    off += c;
  }
  __syncthreads();
  // the table and the non-empty (kind, cube) list written (kind, cube)-consecutive across the lanes
  // (each lane's own run of entries would scatter every store): kind | cube << 1 | (valid + 1) << 14
  // (all passes at once: the non-empty entries ranked by wave ballots, the (pass, wave) counts
  // prefixed by each wave in x order — two barriers instead of three per pass)
  int* items = b.citems + (size_t)p * 2 * kCubeNum;
  constexpr int NW = NT / 64;
  static_assert(NW <= 64, "one count per lane");
  __shared__ int icnt[E][NW];
  const int lane = lane_id(), w = tid >> 6;
  int iex[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int x = e * NT + tid;
    int n = 0;
    if (x < N) {
      const int kind = x / kCubeNum, s = x % kCubeNum, o = nn[x];
      n = (x + 1 < N ? nn[x + 1] : run) - o;
      nw[s * 4 + 2 * kind] = o;
      nw[s * 4 + 1 + 2 * kind] = n;
    }
    const uint64_t m = __ballot(n > 0);
    iex[e] = n > 0 ? __popcll(m & lanemask_lt()) : -1;
    if (lane == 0) icnt[e][w] = __popcll(m);
  }
  __syncthreads();
  int nitems = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int c = lane < NW ? icnt[e][lane] : 0;
    const int incl = wave_incl_scan_x(c);
    const int base = nitems + __shfl(incl - c, w, 64);
    if (iex[e] >= 0) {
      const int x = e * NT + tid;
      items[base + iex[e]] = (x / kCubeNum) | ((x % kCubeNum) << 1) | (((int)vidx[x % kCubeNum] + 1) << 14);
    }
    nitems += __shfl(incl, NW - 1, 64);
  }
  vpts = block_reduce<NT>(vpts, scratch, [](int a, int c) { return a + c; });
  if (tid == 0) {
    b.nitems[p] = nitems;
    b.istate[(size_t)p * kMpStateInts + kMiValidPts] = vpts;
    if (run > b.map_cap) b.istate[(size_t)p * kMpStateInts + kMiErr] |= ERR_CAP_MAP;
  }
}

__global__ __launch_bounds__(256) void k_mp_compact_copy(MpBuffers b) {
  const int p = blockIdx.y;
  const int err = b.istate[(size_t)p * kMpStateInts + kMiErr];
  if (err & ERR_CAP_MAP) return;
  const int* old = slot_table(b, b.pool_cur, p);
  const int* nw = slot_table(b, 1 - b.pool_cur, p);
  const float4* pool = b.pool + ((size_t)b.pool_cur * b.P + p) * b.map_cap;
  float4* npool = b.pool + ((size_t)(1 - b.pool_cur) * b.P + p) * b.map_cap;
  const int* ao = b.app_off + (size_t)p * kCubeNum * 2;
  const float4* app = b.app + (size_t)p * b.cap_stack;
  const int* items = b.citems + (size_t)p * 2 * kCubeNum;
  const int nitems = b.nitems[p];
  for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
    const int code = items[it];
    const int kind = code & 1, s = (code >> 1) & 8191, v = (code >> 14) - 1;
    const int n = nw[s * 4 + 1 + 2 * kind];
    const int dst = nw[s * 4 + 2 * kind];
    if (v >= 0) {
      const int b0 = b.vseg_b[p * 2 * kMaxValid + kind * kMaxValid + v];
      for (int t = threadIdx.x; t < n; t += 256) npool[dst + t] = b.vout[b0 + t];
    } else {
      const int nold = old[s * 4 + 1 + 2 * kind], off = old[s * 4 + 2 * kind];
      for (int t = threadIdx.x; t < n; t += 256)
        npool[dst + t] = t < nold ? pool[off + t] : app[ao[s * 2 + kind] + (t - nold)];
    }
  }
}

// k_mp_register workgroups per problem
#ifndef LOAM_REG_WG
#define LOAM_REG_WG 8  // (1024 problems, k_mp_register ms/step with a per-lane end_rot: 64 -> 1.02, 32 -> 0.77, 16 -> 0.61; with end_rot_wave: 16 -> 0.52, 8 -> 0.50, 4 -> 0.51)
#endif
constexpr int kMpRegWg = LOAM_REG_WG;
__global__ __launch_bounds__(256) void k_mp_register(MpBuffers b, MpInput in) {
  const int p = blockIdx.y;
  const loampose::MapRot r = rot_load(b, p);
  const int n = min(in.nfull[p * in.nfull_stride], b.capS);
  if (in.end_mode) {  // odometry's TransformToEnd of the raw cloud first (k_od_end's, :875-891)
    float t[6] = {0, 0, 0, 0, 0, 0};
    loampose::Imu imu = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (in.end_mode == 2) {
      const float* st = in.end_state + (size_t)p * kOdStateFloats;
      for (int k = 0; k < 6; ++k) t[k] = st[k];
      const float* q = st + kOdImu;
      imu.pitchStart = q[0]; imu.yawStart = q[1]; imu.rollStart = q[2];
      imu.pitchLast = q[3]; imu.yawLast = q[4]; imu.rollLast = q[5];
      imu.shiftX = q[6]; imu.shiftY = q[7]; imu.shiftZ = q[8];
      imu.veloX = q[9]; imu.veloY = q[10]; imu.veloZ = q[11];
    }
    const loampose::EndRot er = loampose::end_rot_wave(t, imu);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
      const float4 a = loampose::transform_to_end(t, imu, er, in.full[(size_t)p * in.full_stride + i], in.end_mode == 1);
      b.reg[(size_t)p * b.capS + i] = loampose::point_to_map(r, a);
    }
  } else {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
      b.reg[(size_t)p * b.capS + i] = loampose::point_to_map(r, in.full[(size_t)p * in.full_stride + i]);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) b.nreg[p] = n;
}

}  // namespace

// ---------------------------------------------------------------- host side
hipError_t mp_alloc(MpBuffers& b, int P, int R, int cap_pts, int map_cap, int max_iter) {
  DevAlloc A;
  b.P = P;
  b.capC = kLessSharpPerRing * R;
  b.capS = cap_pts;
  b.cap_stack = b.capC + b.capS;
  b.map_cap = map_cap;
  b.max_iter = max_iter;
  b.tmax = next_pow2(map_cap) > (1 << 20) ? (1 << 20) : next_pow2(map_cap);
  if (b.tmax < 64) b.tmax = 64;  // >= 64 buckets: a 3x3x3 search never lists a bucket twice (cell_hash)
  b.pool_cur = 0;
  const size_t Pm = (size_t)P * map_cap, Ps = (size_t)P * b.cap_stack;
  A(&b.state, (size_t)P * kMpStateFloats * sizeof(float));
  A(&b.istate, (size_t)P * kMpStateInts * sizeof(int));
  A(&b.slots, (size_t)2 * P * kCubeNum * 4 * sizeof(int));
  A(&b.pool, 2 * Pm * sizeof(float4));
  A(&b.valid, (size_t)P * kMaxValid * sizeof(int));
  A(&b.vpre, (size_t)P * (kMaxValid + 1) * 2 * sizeof(int));
  A(&b.inC, (size_t)P * b.capC * sizeof(float4));
  A(&b.inS, (size_t)P * b.capS * sizeof(float4));
  A(&b.inF, (size_t)P * b.capS * sizeof(float4));
  A(&b.in_n, (size_t)P * 3 * sizeof(int));
  A(&b.in_pose, (size_t)P * 6 * sizeof(float));
  A(&b.stack2, Ps * sizeof(float4));
  A(&b.stack, Ps * sizeof(float4));
  A(&b.nstack, (size_t)P * 2 * sizeof(int));
  A(&b.from, Pm * sizeof(float4));
  A(&b.hC_start, (size_t)P * (b.tmax + 1) * sizeof(int));
  A(&b.hS_start, (size_t)P * (b.tmax + 1) * sizeof(int));
  A(&b.hC_rec, (size_t)P * b.tmax * sizeof(uint32_t));
  A(&b.hS_rec, (size_t)P * b.tmax * sizeof(uint32_t));
  // bucket counters: one set per cloud kind for small batches, whose two builds run together
  A(&b.h_fill, (size_t)2 * P * b.tmax * sizeof(int));  // (corner, surf: built concurrently)
  A(&b.hC_T, (size_t)P * sizeof(int));
  A(&b.hS_T, (size_t)P * sizeof(int));
  A(&b.hC_pts, Pm * sizeof(float4));
  A(&b.hS_pts, Pm * sizeof(float4));
  A(&b.nfrom, (size_t)P * 2 * sizeof(int));
  A(&b.q_ok, Ps * sizeof(int8_t));
  A(&b.q_cf, Ps * sizeof(float4));
  A(&b.q_nn, Ps * 2 * sizeof(int4));
  A(&b.citems, (size_t)P * 2 * kCubeNum * sizeof(int));
  A(&b.nitems, (size_t)P * sizeof(int));
  A(&b.q_fit, Ps * 4 * sizeof(float4));
  A(&b.app_cnt, (size_t)P * kCubeNum * 2 * sizeof(int));
  A(&b.app_off, (size_t)P * kCubeNum * 2 * sizeof(int));
  A(&b.app, Ps * sizeof(float4));
  A(&b.vin, Pm * sizeof(float4));
  A(&b.vout, Pm * sizeof(float4));
  A(&b.vseg_b, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vseg_e, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vseg_cnt, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vseg_leaf, (size_t)P * 2 * kMaxValid * sizeof(float));
  A(&b.sseg_b, (size_t)P * 2 * sizeof(int));
  A(&b.sseg_e, (size_t)P * 2 * sizeof(int));
  A(&b.sseg_cnt, (size_t)P * 2 * sizeof(int));
  A(&b.sseg_leaf, (size_t)P * 2 * sizeof(float));
  const size_t vgn = Pm > Ps ? Pm : Ps;
  A(&b.vg_k, vgn * sizeof(uint32_t));
  A(&b.vg_k2, vgn * sizeof(uint32_t));
  A(&b.vg_v, vgn * sizeof(uint32_t));
  A(&b.vg_v2, vgn * sizeof(uint32_t));
  A(&b.vg_l0, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vg_l1, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vg_lin, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vg_cnt, 4 * sizeof(int));
  A(&b.vg_mlist, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vseg_nold, (size_t)P * 2 * kMaxValid * sizeof(int));
  A(&b.vseg_skip, (size_t)P * 2 * kMaxValid * sizeof(int));
  // the stack job's big-segment split: 2P parents x 16 sub-segments, points / outputs like the stacks
  b.vgs.npar = 2 * P;
  A(&b.vgs.pts, Ps * sizeof(float4));
  A(&b.vgs.out, Ps * sizeof(float4));
  A(&b.vgs.begin, (size_t)P * 32 * sizeof(int));
  A(&b.vgs.end, (size_t)P * 32 * sizeof(int));
  A(&b.vgs.out_count, (size_t)P * 32 * sizeof(int));
  A(&b.vgs.leaf, (size_t)P * 32 * sizeof(float));
  A(&b.vgs.frame, (size_t)P * 32 * sizeof(VgFrame));
  A(&b.vgs.lists[0], (size_t)P * 32 * sizeof(int));
  A(&b.vgs.lists[1], (size_t)P * 32 * sizeof(int));
  A(&b.vgs.counts, 4 * sizeof(int));
  A(&b.vgs.ilist, (size_t)P * 32 * sizeof(int));
  A(&b.reg, (size_t)P * b.capS * sizeof(float4));
  A(&b.part, (size_t)P * std::max(kMpSmallGrid, kMpFitGridMax) * 28 * sizeof(double));
  A(&b.rot, (size_t)P * 6 * sizeof(double));
  A(&b.done, (size_t)P * sizeof(int));
  A(&b.ls_part, (size_t)2 * kMpSmallGrid * 28 * sizeof(double));
  A(&b.ls_flag, (size_t)kMpSmallGrid * sizeof(unsigned long long));
  A(&b.ls_epoch, sizeof(unsigned long long));
  A(&b.nreg, (size_t)P * sizeof(int));
  if (A.err == hipSuccess) A.err = mp_reset(b, nullptr);
  if (A.err == hipSuccess) A.err = hipMemset(b.ls_flag, 0, (size_t)kMpSmallGrid * sizeof(unsigned long long));
  if (A.err == hipSuccess) A.err = hipMemset(b.ls_epoch, 0, sizeof(unsigned long long));
  if (A.err == hipSuccess) A.err = hipDeviceSynchronize();
  if (A.err != hipSuccess) mp_free(b);
  return A.err;
}

void mp_free(MpBuffers& b) {
  void* ptrs[] = {b.state, b.istate, b.slots, b.pool, b.valid, b.vpre, b.inC, b.inS, b.inF, b.in_n, b.in_pose,
                  b.stack2, b.stack, b.nstack, b.from, b.hC_start, b.hS_start, b.hC_rec, b.hS_rec, b.h_fill, b.hC_T, b.hS_T,
                  b.hC_pts, b.hS_pts, b.nfrom, b.q_ok, b.q_cf, b.q_nn, b.q_fit, b.citems, b.nitems, b.app_cnt, b.app_off, b.app, b.vin, b.vout,
                  b.vseg_b, b.vseg_e, b.vseg_cnt, b.vseg_leaf, b.sseg_b, b.sseg_e, b.sseg_cnt, b.sseg_leaf,
                  b.vg_k, b.vg_k2, b.vg_v, b.vg_v2, b.vg_l0, b.vg_l1, b.vg_lin, b.vg_cnt, b.reg, b.nreg, b.part, b.done, b.rot,
                  b.vg_mlist, b.vseg_nold, b.vseg_skip, b.ls_part, b.ls_flag, b.ls_epoch, b.vgs.pts, b.vgs.out,
                  b.vgs.begin, b.vgs.end, b.vgs.out_count, b.vgs.leaf, b.vgs.frame, b.vgs.lists[0], b.vgs.lists[1],
                  b.vgs.counts, b.vgs.ilist};
  if (b.upd_pending && b.upd_done) (void)hipEventSynchronize(b.upd_done);
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (b.upd_fork) (void)hipEventDestroy(b.upd_fork);
  if (b.upd_done) (void)hipEventDestroy(b.upd_done);
  b = MpBuffers();
}

__global__ void k_mp_reset(MpBuffers b) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= b.P) return;
  int* ist = b.istate + (size_t)p * kMpStateInts;
  ist[kMiCenW] = 10; ist[kMiCenH] = 5; ist[kMiCenD] = 10;  // :64-66
}

hipError_t mp_reset(MpBuffers& b, hipStream_t st) {
  mp_wait_update(b, st);
  b.pool_cur = 0;
  hipError_t e = hipMemsetAsync(b.state, 0, (size_t)b.P * kMpStateFloats * sizeof(float), st);
  if (e == hipSuccess) e = hipMemsetAsync(b.done, 0, (size_t)b.P * sizeof(int), st);
  if (e == hipSuccess) e = hipMemsetAsync(b.istate, 0, (size_t)b.P * kMpStateInts * sizeof(int), st);
  if (e == hipSuccess) e = hipMemsetAsync(b.slots, 0, (size_t)2 * b.P * kCubeNum * 4 * sizeof(int), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_mp_reset, dim3((b.P + 255) / 256), dim3(256), 0, st, b);
  return hipGetLastError();
}

void mp_wait_update(MpBuffers& b, hipStream_t st) {
  if (!b.upd_pending) return;
  b.note(hipStreamWaitEvent(st, b.upd_done, 0));
  b.upd_pending = false;
}

void mp_frame(MpBuffers& b, const MpInput& in, hipStream_t st, Prof* prof, bool map_empty,
              const std::function<void()>& before_register, int stack_max, const SideStream* side,
              hipStream_t defer) {
  const int P = b.P;
  auto mark = [&](const char* n) { if (prof) prof->mark(n); };
  mp_wait_update(b, st);  // (the previous frame's map update, when it was deferred)
  hipLaunchKernelGGL(k_mp_prepare, dim3(P), dim3(kMpThreads), 0, st, b, in);
  mark("k_mp_prepare");
  hipLaunchKernelGGL(k_mp_stack, dim3(16, P), dim3(256), 0, st, b, in);
  mark("k_mp_stack");
  if (side && side->inputs_read) b.note(hipEventRecord(side->inputs_read, st));  // (in.corner / in.surf read)
  VgJob js = vg_job(b);
  js.in = b.stack2; js.out = b.stack; js.begin = b.sseg_b; js.end = b.sseg_e; js.leaf = b.sseg_leaf;
  js.out_count = b.sseg_cnt; js.nseg = 2 * P; js.total = P * b.cap_stack;
  // two large segments per instance (the fused 12288-point kernel); when the host knows both fit
  // (streaming), the cascade's finish is not enqueued
  // (k_mp_stack zeroed the cascade's list counters)
  js.zeroed = true;
  // (the cascade's first kernel takes 12288 points for a few instances, 2048 for batches)
  const bool fits = stack_max >= 0 && stack_max <= (P <= 4 ? 12288 : 2048);
  // batches: the corner stacks (<= 120 points per ring) take the 2048-point kernel, the surf
  // stacks the 12288-point one; a few instances: one 12288-point launch.  With a side stream it
  // runs there, beside the FromMap gather and the map hash builds (which read only the store)
  const bool fork = side && side->st && !prof && !map_empty;
  if (fork) {
    b.note(hipEventRecord(side->fork[0], st));
    b.note(hipStreamWaitEvent(side->st, side->fork[0], 0));
  }
  // (vg_split 1: the split takes the segments beyond the first kernel when a sweep can fill several
  // LDS-tier segments (HDL-64E: 64 problems 0.56 -> 0.49 ms/step), else only those beyond the LDS
  // kernels (VLP-16 at 128 / 1024 problems: splitting beyond the first kernel 0.24 -> 0.32 ms/step))
  const bool split_early = b.tune.vg_split == 3 || (b.tune.vg_split == 1 && b.capS > 4 * 16384);
  b.note(vg_run<kVgStack>(js, fork ? side->st : st, P <= 4 ? 12288 : 2048, !fits, /*tier2_idx=*/true,
                          b.tune.vg_split ? &b.vgs : nullptr, split_early));
  if (fork) b.note(hipEventRecord(side->join[0], side->st));
  mark("vg_stack");
  hipLaunchKernelGGL(k_mp_gather, dim3(32, P), dim3(256), 0, st, b);
  mark("k_mp_gather");
  HashJob hc;
  hc.pts = b.from; hc.pts_stride = b.map_cap; hc.pts_off = nullptr; hc.pts_off_stride = 0;
  hc.count = b.nfrom; hc.count_stride_bytes = 2 * sizeof(int);
  hc.start = b.hC_start; hc.fill = b.h_fill; hc.out = b.hC_pts; hc.tsize = b.hC_T; hc.tmax = b.tmax;
  hc.inv_h = 1.0f;
  hc.shift = 0;  // the 5-NN search scans whole buckets: keep them to single cells
  hc.chunks = nullptr;
  hc.rec = b.hC_rec;
  HashJob hs = hc;
  hs.rec = b.hS_rec;
  hs.pts_off = b.nfrom; hs.pts_off_stride = 2;
  hs.count = b.nfrom + 1; hs.start = b.hS_start; hs.out = b.hS_pts; hs.tsize = b.hS_T;
  hs.fill = b.h_fill + (size_t)P * b.tmax;  // (the two indexes are built in one launch / concurrently)
  hash_build_pair(hc, hs, P, st, false);
  mark("k_hash_build_map");
  if (fork) b.note(hipStreamWaitEvent(st, side->join[0], 0));
  hipLaunchKernelGGL(k_mp_lm_begin, dim3((P + 255) / 256), dim3(256), 0, st, b);
  // workgroups per instance: all the stack's queries at once for a few instances; for large
  // batches about one pass over a VLP-16 stack (bigger stacks loop), fewer idle workgroups
  const int gq = std::min(P >= 64 ? 24 : 64, (b.cap_stack + kMpQueryThreads - 1) / kMpQueryThreads);
  // an empty map store (the first frame after a reset) cannot run the L-M (:706): no launches
  // one instance (streaming): the whole L-M loop as one persistent launch (tuning mp_persist)
  const int gls = P == 1 && !map_empty && b.tune.mp_persist ? mp_lm_stream_grid() : 0;
  if (gls > 0) {
    hipLaunchKernelGGL(k_mp_lm_stream, dim3(gls), dim3(kMpQueryThreads), 0, st, b);
    mark("k_mp_lm_stream");
  }
  for (int it = 0; it < (map_empty || gls > 0 ? 0 : b.max_iter); ++it) {
    if (P <= b.tune.mp_small_max) {  // small batches: one launch per iteration
      hipLaunchKernelGGL(k_mp_lm_small, dim3(kMpSmallGrid, P), dim3(kMpQueryThreads), 0, st, b);
      mark("k_mp_lm_small");
      continue;
    }
    // (P >= 512: 64 workgroups, two passes per lane over a VLP-16 stack; round 6 at 1024 problems:
    // 12.28-12.32 -> 12.20-12.23 ms/step against 96; at 128 the one-pass 96 stays best)
    const int gfit_auto = P >= 512 ? 64 : gq * (kMpQueryThreads / kMpFitThreads);
    const int gfit = std::min(kMpFitGridMax, b.tune.fit_wg > 0 ? b.tune.fit_wg : gfit_auto);
    // search + fit (+ step) in one launch (round 3's separate k_mp_nn / k_mp_fit launches, and 2 / 4
    // lanes per query, measured slower and were removed in round 6)
    const bool fused = P <= b.tune.mp_fused_max;
    if (fused && prof) hipLaunchKernelGGL((k_mp_nnfit<true, true>), dim3(gfit, P), dim3(kMpFitThreads), 0, st, b);
    else if (fused) hipLaunchKernelGGL((k_mp_nnfit<true, false>), dim3(gfit, P), dim3(kMpFitThreads), 0, st, b);
    else if (prof) hipLaunchKernelGGL((k_mp_nnfit<false, true>), dim3(gfit, P), dim3(kMpFitThreads), 0, st, b);
    else hipLaunchKernelGGL((k_mp_nnfit<false, false>), dim3(gfit, P), dim3(kMpFitThreads), 0, st, b);
    mark("k_mp_nnfit");
    if (!fused) {
      hipLaunchKernelGGL(k_mp_iter<kMpThreads>, dim3(P), dim3(kMpThreads), 0, st, b);
      mark("k_mp_iter");
    }
  }
  hipLaunchKernelGGL(k_mp_lm_end, dim3((P + 255) / 256), dim3(256), 0, st, b);
  // the registration reads only the final pose and the full cloud: beside the insertion with a
  // side stream (the batch: no before_register hook)
  const bool reg_side = fork && !before_register && !defer;
  // defer: the map update on the other stream, forked here; the registration stays on st
  hipStream_t us = st;
  if (defer) {
    if (!b.upd_fork) b.note(hipEventCreateWithFlags(&b.upd_fork, hipEventDisableTiming));
    if (!b.upd_done) b.note(hipEventCreateWithFlags(&b.upd_done, hipEventDisableTiming));
    b.note(hipEventRecord(b.upd_fork, st));
    b.note(hipStreamWaitEvent(defer, b.upd_fork, 0));
    us = defer;
  }
  if (reg_side) {
    b.note(hipEventRecord(side->fork[1], st));
    b.note(hipStreamWaitEvent(side->st, side->fork[1], 0));
    hipLaunchKernelGGL(k_mp_register, dim3(kMpRegWg, P), dim3(256), 0, side->st, b, in);
    b.note(hipEventRecord(side->join[1], side->st));
  }
  // insertion + per-valid-cube downsampling into the other pool
  // a few instances: 1024 threads per instance (the per-instance serial parts are the cost)
  // 1024 threads per instance also for batches (k_mp_insert 0.40 -> 0.25 ms/step at batch 1024 against 256)
  hipLaunchKernelGGL(k_mp_insert<1024>, dim3(P), dim3(1024), 0, us, b, (int*)b.vg_k, (int*)b.vg_v);
  mark("k_mp_insert");
  hipLaunchKernelGGL(k_mp_vseg, dim3(P), dim3(kMpThreads), 0, us, b);
  hipLaunchKernelGGL(k_mp_vcopy, dim3(32, P), dim3(256), 0, us, b);
  mark("k_mp_vseg_vcopy");
  VgJob jv = vg_job(b);
  jv.in = b.vin; jv.out = b.vout; jv.begin = b.vseg_b; jv.end = b.vseg_e; jv.leaf = b.vseg_leaf;
  jv.out_count = b.vseg_cnt; jv.nseg = 2 * kMaxValid * P; jv.total = P * b.map_cap;
  // only the non-empty segments, listed by k_mp_vseg (k_mp_lm_end zeroed the counters)
  jv.list = b.vg_lin; jv.list_n = b.vg_cnt + 2; jv.zeroed = true;
  if (b.tune.vg_merge) {  // long cube segments with a short tail first (k_vg_merge), the rest by the cascade
    jv.nold = b.vseg_nold; jv.mlist = b.vg_mlist; jv.mlist_n = b.vg_cnt + 3; jv.skip = b.vseg_skip;
    // (its segments are rare: a small grid whose workgroups leave at once when the list is short)
    hipLaunchKernelGGL((k_vg_merge<1024, kVgMergeNew>), dim3(std::min(2 * kMaxValid * P, 32)), dim3(1024), 0, us, jv);
  }
  // 2 x 125 cube segments per instance, most of them small: batches start with the 2048-point
  // kernel (many workgroups per CU); a few instances with the 12288-point one (one launch)
  b.note(vg_run<kVgCubes>(jv, us, P <= 4 ? 12288 : 2048));
  mark("vg_cubes");
  hipLaunchKernelGGL(k_mp_compact_table<1024>, dim3(P), dim3(1024), 0, us, b);
  hipLaunchKernelGGL(k_mp_compact_copy, dim3(64, P), dim3(256), 0, us, b);
  mark("k_mp_compact");
  if (defer) {
    b.note(hipEventRecord(b.upd_done, us));
    b.upd_pending = true;
  }
  if (before_register) before_register();
  if (reg_side) {
    b.note(hipStreamWaitEvent(st, side->join[1], 0));
  } else {
    hipLaunchKernelGGL(k_mp_register, dim3(kMpRegWg, P), dim3(256), 0, st, b, in);
    mark("k_mp_register");
  }
  b.pool_cur = 1 - b.pool_cur;
}

template <typename Hook>
int mp_stream_run(MpBuffers& b, hipStream_t st, const MpInput& in, const int* n, loam_pose6* aft, loam_pose6* bef,
                  loam_cloud_out* registered, loam_stats* stats, std::string& err, Staging& pin, const StreamIo& io,
                  bool* updated, Hook hook, hipStream_t defer);

int mp_stream_frame(MpBuffers& b, hipStream_t st, const loam_pose6& odom_sum, const loam_cloud_out& corner,
                    const loam_cloud_out& surf, const loam_cloud_out& full, loam_pose6* aft, loam_pose6* bef,
                    loam_cloud_out* registered, loam_stats* stats, std::string& err, Staging& pin, const StreamIo& io,
                    const float* imu_rp, bool* updated, hipStream_t st2, hipEvent_t ev2, hipStream_t defer) {
  if (corner.count > (uint32_t)b.capC || surf.count > (uint32_t)b.capS || full.count > (uint32_t)b.capS) {
    err = "mapping input cloud exceeds capacity";
    return LOAM_E_CAPACITY;
  }
  if ((corner.count && !corner.pts) || (surf.count && !surf.pts) || (full.count && !full.pts)) {
    err = "mapping input cloud pts is null";
    return LOAM_E_INVAL;
  }
  // host inputs: [0..2] counts, [4..9] pose, [10..11] IMU (roll, pitch), [12] IMU flag, to the
  // device in one k_xfer launch; downloads through io.xb (mp_stream_run)
  int mi[16];
  int* n = mi;
  n[0] = (int)corner.count; n[1] = (int)surf.count; n[2] = (int)full.count;
  std::memcpy(mi + 4, &odom_sum, 6 * sizeof(float));
  const float rp[2] = {imu_rp ? imu_rp[0] : 0.0f, imu_rp ? imu_rp[1] : 0.0f};
  std::memcpy(mi + 10, rp, sizeof(rp));
  mi[12] = imu_rp ? 1 : 0;
  pin.reset();
  // room for all three clouds now: the full cloud is staged later, while the kernels run
  hipError_t ue = pin.reserve((size_t)n[0] + n[1] + n[2], st);
  if (ue == hipSuccess) ue = pin.up(st, b.inC, corner.pts, (size_t)n[0]);
  if (ue == hipSuccess) ue = pin.up(st, b.inS, surf.pts, (size_t)n[1]);
  // only k_mp_register reads the full cloud: with a second stream its staging copy and DMA
  // overlap the frame's kernels (enqueued just before k_mp_register)
  const bool late = st2 != nullptr && n[2] > 0;
  if (ue == hipSuccess && !late) ue = pin.up(st, b.inF, full.pts, (size_t)n[2]);
  if (ue == hipSuccess) {
    Xfer xp;
    xp.put(b.in_n, n, 3 * sizeof(int));
    xp.put(b.in_pose, mi + 4, 6 * sizeof(float));
    xp.put(b.state + kMpImuRP, mi + 10, 2 * sizeof(float));
    xp.put(b.istate + kMiImu, mi + 12, sizeof(int));
    ue = xfer_launch(xp, st);
  }
  if (ue != hipSuccess) {
    err = std::string("mapping upload: ") + hipGetErrorString(ue);
    return LOAM_E_HIP;
  }
  MpInput in;
  in.corner = b.inC; in.surf = b.inS; in.full = b.inF;
  in.corner_stride = b.capC; in.surf_stride = b.capS; in.full_stride = b.capS;
  in.ncorner = b.in_n; in.nsurf = b.in_n + 1; in.nfull = b.in_n + 2;
  in.ncorner_stride = in.nsurf_stride = in.nfull_stride = 3;
  in.pose = b.in_pose; in.pose_stride = 6;
  return mp_stream_run(b, st, in, n, aft, bef, registered, stats, err, pin, io, updated, [&]() {
    if (!late) return hipSuccess;
    hipError_t le = pin.up(st2, b.inF, full.pts, (size_t)n[2]);
    if (le == hipSuccess) le = hipEventRecord(ev2, st2);
    if (le == hipSuccess) le = hipStreamWaitEvent(st, ev2, 0);
    return le;
  }, defer);
}

// the device-resident chain (loam_chain_sweep): the clouds are already on the device (odometry's
// published Last / full-end buffers, src, with device counts); n3: their counts on the host
int mp_stream_frame_dev(MpBuffers& b, hipStream_t st, const loam_pose6& odom_sum, const MpInput& src, const int* n3,
                        loam_pose6* aft, loam_pose6* bef, loam_cloud_out* registered, loam_stats* stats,
                        std::string& err, Staging& pin, const StreamIo& io, const float* imu_rp, bool* updated,
                        hipStream_t defer) {
  if (n3[0] > b.capC || n3[1] > b.capS || n3[2] > b.capS) {
    err = "mapping input cloud exceeds capacity";
    return LOAM_E_CAPACITY;
  }
  // as mp_stream_frame: the pose, the IMU (roll, pitch) and flag in one k_xfer launch
  const float rp[2] = {imu_rp ? imu_rp[0] : 0.0f, imu_rp ? imu_rp[1] : 0.0f};
  const int flag = imu_rp ? 1 : 0;
  Xfer xp;
  xp.put(b.in_pose, &odom_sum, 6 * sizeof(float));
  xp.put(b.state + kMpImuRP, rp, sizeof(rp));
  xp.put(b.istate + kMiImu, &flag, sizeof(int));
  const hipError_t ue = xfer_launch(xp, st);
  if (ue != hipSuccess) {
    err = std::string("mapping upload: ") + hipGetErrorString(ue);
    return LOAM_E_HIP;
  }
  MpInput in = src;
  in.pose = b.in_pose;
  in.pose_stride = 6;
  return mp_stream_run(b, st, in, n3, aft, bef, registered, stats, err, pin, io, updated,
                       []() { return hipSuccess; }, defer);
}

// the frame's kernels on `in` and the downloads (both stream entry points); hook: called just
// before k_mp_register (the late full-cloud staging); defer: the map update's stream (mp_frame),
// nullptr = in order on st
template <typename Hook>
int mp_stream_run(MpBuffers& b, hipStream_t st, const MpInput& in, const int* n, loam_pose6* aft, loam_pose6* bef,
                  loam_cloud_out* registered, loam_stats* stats, std::string& err, Staging& pin, const StreamIo& io,
                  bool* updated, Hook hook, hipStream_t defer) {
  const hipEvent_t e0 = io.e0, e1 = io.e1;
  hipError_t le = hipEventRecord(e0, st);
  mp_frame(b, in, st, nullptr, false, [&]() {
    if (le != hipSuccess) return;
    le = hook();
  }, std::max(n[0], n[1]), nullptr, defer);
  if (le == hipSuccess) le = hipEventRecord(e1, st);
  // a deferred update's valid-point count (stats) into the mapped host block after it, one slot
  // per frame parity: this call reads the previous frame's (complete: this frame's kernels on st
  // waited for that update), while this frame's may still be writing the other slot
  const bool deferred = defer && b.upd_pending;
  if (deferred && le == hipSuccess) {
    Xfer xg;
    xg.get(io.xb.d + kXferMpUpd + 4 * (1 - b.pool_cur), b.istate + kMiValidPts, sizeof(int));
    le = xfer_launch(xg, defer);
    if (le == hipSuccess) le = hipEventRecord(b.upd_done, defer);
  }
  // state (kMpStateFloats), istate (kMpStateInts), nreg into the mapped host block, one launch
  static_assert(kXferMp + 4 * (kMpStateFloats + kMpStateInts + 1) <= kXferMpUpd, "mapping transfer region");
  static_assert(kXferMpUpd + 8 <= kXferBytes, "deferred valid-point slots");
  const float* sf = (const float*)(io.xb.h + kXferMp);
  const int* si = (const int*)(io.xb.h + kXferMp) + kMpStateFloats;
  const int* pnreg = si + kMpStateInts;
  {
    Xfer xg;
    char* d = io.xb.d + kXferMp;
    xg.get(d, b.state, kMpStateFloats * sizeof(float));
    xg.get(d + kMpStateFloats * 4, b.istate, kMpStateInts * sizeof(int));
    xg.get(d + (kMpStateFloats + kMpStateInts) * 4, b.nreg, sizeof(int));
    le = le == hipSuccess ? xfer_launch(xg, st) : le;
  }
  hipError_t he = hipGetLastError();
  if (he == hipSuccess) he = hipStreamSynchronize(st);
  const int nreg = *pnreg;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  if (he == hipSuccess) he = b.take_error();
  if (he == hipSuccess) he = le;
  if (he != hipSuccess) {
    err = std::string("mapping: ") + hipGetErrorString(he);
    return LOAM_E_HIP;
  }
  if (si[kMiErr]) {
    err = "mapping capacity exceeded (map store / stack)";
    return LOAM_E_CAPACITY;
  }
  std::memcpy(aft, sf + kMpAft, sizeof(loam_pose6));
  std::memcpy(bef, sf + kMpBef, sizeof(loam_pose6));
  if (updated) *updated = si[kMiLmRan] != 0;
  int rc = LOAM_OK;
  if (registered) {
    if ((uint32_t)nreg > registered->capacity) {
      registered->count = (uint32_t)nreg;
      err = "registered cloud capacity too small";
      rc = LOAM_E_CAPACITY;
    } else {
      registered->count = (uint32_t)nreg;
      pin.reset();
      he = pin.down(st, registered->pts, b.reg, (size_t)nreg);
      if (he == hipSuccess) he = hipStreamSynchronize(st);
      if (he != hipSuccess) {
        err = std::string("registered cloud download: ") + hipGetErrorString(he);
        return LOAM_E_HIP;
      }
      pin.finish();
    }
  }
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->mp_iters = si[kMiIters];
    stats->mp_rows_sum = (uint64_t)si[kMiRows];
    stats->mp_stack = (uint64_t)(si[kMiStackC] + si[kMiStackS]);
    stats->mp_stack_iters = (uint64_t)si[kMiIters] * (si[kMiStackC] + si[kMiStackS]);
    stats->mp_fits = (uint64_t)si[kMiFits];
    stats->mp_map_points = (uint64_t)(si[kMiFromC] + si[kMiFromS]);
    // (a deferred update: the previous frame's map, this frame's is not counted yet)
    stats->mp_map_valid_points =
        (uint64_t)(deferred ? *(const int*)(io.xb.h + kXferMpUpd + 4 * b.pool_cur) : si[kMiValidPts]);
    stats->mp_degenerate_steps = (uint64_t)si[kMiDegSteps];
    stats->mp_grid_shifts = (uint64_t)si[kMiShifts];
    stats->mp_nn_candidates = (uint64_t)(uint32_t)si[kMiNnCand];
    stats->mp_nn_cells = (uint64_t)(uint32_t)si[kMiNnCells];
    stats->ms_mp = ms;
  }
  return rc;
}

// /laser_cloud_surround input (:1042-1047): every in-bounds cube of the 5x5x5 neighbourhood of the
// frame's centre cube (laserCloudSurroundInd, :617-670, FOV test or not) in (i, j, k) loop order,
// each cube's corner points then its surf points, from the store the frame left; one VoxelGrid
// segment (leaf 0.2, downSizeFilterCorner) over vin.
__global__ __launch_bounds__(256) void k_mp_surround(MpBuffers b) {
  const int tid = threadIdx.x;
  if (tid == 0) { b.vg_cnt[0] = 0; b.vg_cnt[1] = 0; }  // (its VoxelGrid's lists)
  const int* ist = b.istate;
  const int* slots = slot_table(b, b.pool_cur, 0);
  const float4* pool = b.pool + (size_t)b.pool_cur * b.P * b.map_cap;
  __shared__ int sh_ind[kMaxValid], sh_pre[kMaxValid + 1], sh_n;
  if (tid == 0) {
    const int cI = ist[kMiCubeI], cJ = ist[kMiCubeJ], cK = ist[kMiCubeK];
    int n = 0, acc = 0;
    for (int i = cI - 2; i <= cI + 2; ++i)
      for (int j = cJ - 2; j <= cJ + 2; ++j)
        for (int k = cK - 2; k <= cK + 2; ++k) {
          if (!(i >= 0 && i < kCubeW && j >= 0 && j < kCubeH && k >= 0 && k < kCubeD)) continue;
          const int ind = cube_index(i, j, k);
          sh_ind[n] = ind;
          sh_pre[n] = acc;
          acc += slots[ind * 4 + 1] + slots[ind * 4 + 3];
          ++n;
        }
    sh_pre[n] = acc;
    sh_n = n;
    b.vseg_b[0] = 0;
    b.vseg_e[0] = acc;
    b.vseg_leaf[0] = 0.2f;
  }
  __syncthreads();
  const int n = sh_n;
  for (int c = 0; c < n; ++c) {
    const int ind = sh_ind[c], nc = slots[ind * 4 + 1], ns = slots[ind * 4 + 3];
    const int oc = slots[ind * 4 + 0], os = slots[ind * 4 + 2];
    float4* dst = b.vin + sh_pre[c];
    for (int t = tid; t < nc + ns; t += 256) dst[t] = t < nc ? pool[oc + t] : pool[os + (t - nc)];
  }
}

int mp_stream_surround(MpBuffers& b, hipStream_t st, loam_cloud_out* out, std::string& err) {
  mp_wait_update(b, st);  // (the last frame's map update, when deferred)
  hipLaunchKernelGGL(k_mp_surround, dim3(1), dim3(256), 0, st, b);
  VgJob j = vg_job(b);
  j.in = b.vin; j.out = b.vout; j.begin = b.vseg_b; j.end = b.vseg_e; j.leaf = b.vseg_leaf;
  j.out_count = b.vseg_cnt; j.nseg = 1; j.total = b.P * b.map_cap;
  j.zeroed = true;  // (by k_mp_surround)
  b.note(vg_run<kVgSurround>(j, st, 12288));
  int cnt = 0;
  hipError_t he = hipMemcpyAsync(&cnt, b.vseg_cnt, sizeof(int), hipMemcpyDeviceToHost, st);
  if (he == hipSuccess) he = hipStreamSynchronize(st);
  if (he == hipSuccess) he = b.take_error();
  if (he != hipSuccess) {
    err = std::string("surround: ") + hipGetErrorString(he);
    return LOAM_E_HIP;
  }
  if ((uint32_t)cnt > out->capacity) {
    out->count = (uint32_t)cnt;
    err = "surround cloud capacity too small";
    return LOAM_E_CAPACITY;
  }
  out->count = (uint32_t)cnt;
  if (cnt && hipMemcpy(out->pts, b.vout, (size_t)cnt * sizeof(float4), hipMemcpyDeviceToHost) != hipSuccess) {
    err = "surround download failed";
    return LOAM_E_HIP;
  }
  return LOAM_OK;
}

// frame 1 of the batch problem: reset, then prev (the seed's Last[buf]) into the empty store at
// the zero pose.  Reads only what the odometry seeding wrote, so it may run beside od_solve.
void mp_batch_frame1(MpBuffers& b, const OdBuffers& od, int buf, const FeatView& fprev, hipStream_t st, Prof* prof,
                     const SideStream* side) {
  b.note(mp_reset(b, st));
  if (prof) prof->mark("mp_reset");
  MpInput in;
  in.corner = od.lastC + (size_t)buf * od.P * od.capC;
  in.surf = od.lastS + (size_t)buf * od.P * od.capS;
  in.corner_stride = od.capC; in.surf_stride = od.capS;
  in.ncorner = od.nlast + buf * 2; in.nsurf = od.nlast + buf * 2 + 1;
  in.ncorner_stride = 2 * kOdBufs; in.nsurf_stride = 2 * kOdBufs;
  // the full cloud: prev's raw one, TransformToEnd with the zero transform in k_mp_register
  in.full = fprev.full; in.full_stride = fprev.full_stride;
  in.nfull = fprev.nfull_p; in.nfull_stride = fprev.nfull_stride;
  in.end_mode = 1;
  in.pose = nullptr; in.pose_stride = 0;
  mp_frame(b, in, st, prof, /*map_empty=*/true, nullptr, -1, side);
}

// frame 2: cur (TransformToEnd's Last[buf]) with the odometry transformSum
void mp_batch_frame2(MpBuffers& b, const OdBuffers& od, int buf, const FeatView& fcur, hipStream_t st, Prof* prof,
                     const SideStream* side) {
  MpInput in;
  in.corner = od.lastC + (size_t)buf * od.P * od.capC;
  in.surf = od.lastS + (size_t)buf * od.P * od.capS;
  in.corner_stride = od.capC; in.surf_stride = od.capS;
  in.ncorner = od.nlast + buf * 2; in.nsurf = od.nlast + buf * 2 + 1;
  in.ncorner_stride = 2 * kOdBufs; in.nsurf_stride = 2 * kOdBufs;
  // the full cloud: cur's raw one, TransformToEnd with the solved transform in k_mp_register
  in.full = fcur.full; in.full_stride = fcur.full_stride;
  in.nfull = fcur.nfull_p; in.nfull_stride = fcur.nfull_stride;
  in.end_state = od.state; in.end_mode = 2;
  in.pose = od.state + kOdSum; in.pose_stride = kOdStateFloats;
  mp_frame(b, in, st, prof, false, nullptr, -1, side);
}

// per-instance mapping L-M iteration counts of the last frame (loam_batch_iterations)
hipError_t mp_batch_iters(MpBuffers& b, hipStream_t st, int32_t* iters) {
  std::vector<int> si((size_t)b.P * kMpStateInts);
  hipError_t he = hipStreamSynchronize(st);
  if (he == hipSuccess) he = hipMemcpy(si.data(), b.istate, si.size() * sizeof(int), hipMemcpyDeviceToHost);
  if (he == hipSuccess)
    for (int p = 0; p < b.P; ++p) iters[p] = si[(size_t)p * kMpStateInts + kMiIters];
  return he;
}

int mp_batch_download(MpBuffers& b, hipStream_t st, loam_pose6* aft, loam_stats* stats, std::string& err) {
  std::vector<float> sf((size_t)b.P * kMpStateFloats);
  std::vector<int> si((size_t)b.P * kMpStateInts);
  hipError_t he = hipStreamSynchronize(st);
  if (he == hipSuccess) he = b.take_error();
  if (he == hipSuccess) he = hipMemcpy(sf.data(), b.state, sf.size() * sizeof(float), hipMemcpyDeviceToHost);
  if (he == hipSuccess) he = hipMemcpy(si.data(), b.istate, si.size() * sizeof(int), hipMemcpyDeviceToHost);
  if (he != hipSuccess) {
    err = std::string("mapping: ") + hipGetErrorString(he);
    return LOAM_E_HIP;
  }
  for (int p = 0; p < b.P; ++p) {
    const int* q = &si[(size_t)p * kMpStateInts];
    if (q[kMiErr]) {
      err = "mapping capacity exceeded (map store / stack)";
      return LOAM_E_CAPACITY;
    }
    if (aft) std::memcpy(&aft[p], &sf[(size_t)p * kMpStateFloats + kMpAft], sizeof(loam_pose6));
    if (stats) {
      stats->mp_iters += q[kMiIters];
      stats->mp_rows_sum += (uint64_t)q[kMiRows];
      stats->mp_stack += (uint64_t)(q[kMiStackC] + q[kMiStackS]);
      stats->mp_stack_iters += (uint64_t)q[kMiIters] * (q[kMiStackC] + q[kMiStackS]);
      stats->mp_fits += (uint64_t)q[kMiFits];
      stats->mp_map_points += (uint64_t)(q[kMiFromC] + q[kMiFromS]);
      stats->mp_map_valid_points += (uint64_t)q[kMiValidPts];
      stats->mp_degenerate_steps += (uint64_t)q[kMiDegSteps];
      stats->mp_grid_shifts += (uint64_t)q[kMiShifts];
      stats->mp_nn_candidates += (uint64_t)(uint32_t)q[kMiNnCand];
      stats->mp_nn_cells += (uint64_t)(uint32_t)q[kMiNnCells];
    }
  }
  return LOAM_OK;
}

}  // namespace loam

#ifdef LOAM_PHASES
// the phase sums of the last-workgroup kernel of this file (PhaseAcc, dev_common.hpp); diagnostic
// build only (tools/phase_stream.py)
extern "C" int loam_debug_phases_mp(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(loam::g_ph_mp), sizeof(PhaseAcc)) == hipSuccess ? 0 : -1;
}
#endif
