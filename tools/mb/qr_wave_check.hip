// Check of the wave-parallel 6x6 QR solve (dev_common.hpp loamla::qr_solve6_wave) against the
// one-lane qr_solve on random systems: normal equations of random Jacobians at several scales,
// rank-deficient ones (the |R_ii| < eps exit), general matrices, and some with NaN / inf entries.
// Bit-for-bit comparison of x and of the return flag (any NaN matches any NaN).  Then the latency of one call of each on one
// wave (the matrix changed every repetition, so nothing is hoisted).  Built by
// loam_velodyne-1_amd/Makefile; run by tests/test_gpu_waveops.py.  Exit 0 when every result matches.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../loam_velodyne-1_amd/csrc/dev_common.hpp"

__global__ void k_ref(const float* A, const float* b, int n, float* x, int* ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a[36], bb[6], ws[14], xx[6];
  for (int k = 0; k < 36; ++k) a[k] = A[i * 36 + k];
  for (int k = 0; k < 6; ++k) bb[k] = b[i * 6 + k];
  ok[i] = loamla::qr_solve(a, bb, 6, 6, xx, ws) ? 1 : 0;
  for (int k = 0; k < 6; ++k) x[i * 6 + k] = xx[k];
}

__global__ void k_wave(const float* A, const float* b, float* x, int* ok) {
  const int i = blockIdx.x;
  float xx[6];
  const bool r = loamla::qr_solve6_wave(A + i * 36, b + i * 6, xx);
  if (threadIdx.x == 0) {
    ok[i] = r ? 1 : 0;
    for (int k = 0; k < 6; ++k) x[i * 6 + k] = xx[k];
  }
}

template <bool WAVE>
__global__ void k_time(const float* A, const float* b, int reps, float* out) {
  __shared__ float sA[36], sB[6];
  if (threadIdx.x < 36) sA[threadIdx.x] = A[threadIdx.x];
  if (threadIdx.x < 6) sB[threadIdx.x] = b[threadIdx.x];
  __syncthreads();
  float acc = 0.0f;
  for (int r = 0; r < reps; ++r) {
    float xx[6];
    if (WAVE) {
      loamla::qr_solve6_wave(sA, sB, xx);
    } else if (threadIdx.x == 0) {
      float a[36], bb[6], ws[14];
      for (int k = 0; k < 36; ++k) a[k] = sA[k];
      for (int k = 0; k < 6; ++k) bb[k] = sB[k];
      loamla::qr_solve(a, bb, 6, 6, xx, ws);
    }
    if (threadIdx.x == 0) {
      acc += xx[0] + xx[5];
      sA[r % 36] += 1e-9f * acc;  // the next call's matrix depends on this one's result
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  if (threadIdx.x == 0) out[WAVE ? 1 : 0] = acc;
}

int main() {
  const int n = 1 << 15;
  std::mt19937 rng(11);
  std::normal_distribution<float> nd;
  std::uniform_real_distribution<float> ud(0.0f, 1.0f);
  std::vector<float> A((size_t)n * 36), b((size_t)n * 6);
  for (int s = 0; s < n; ++s) {
    float* a = &A[(size_t)s * 36];
    float* r = &b[(size_t)s * 6];
    const int kind = s % 8;
    if (kind < 5) {  // normal equations J^T J, J^T e of rows at a scale
      const int rows = 7 + (int)(ud(rng) * 300);
      const float sc = std::pow(10.0f, -3.0f + 6.0f * ud(rng));
      std::vector<double> AtA(36, 0.0), AtB(6, 0.0);
      const bool deficient = kind == 4;
      for (int k = 0; k < rows; ++k) {
        float j[6];
        for (int c = 0; c < 6; ++c) j[c] = nd(rng) * sc;
        if (deficient) j[5] = j[4];
        const float e = nd(rng) * 0.05f;
        for (int p = 0; p < 6; ++p) {
          for (int q = 0; q < 6; ++q) AtA[p * 6 + q] += (double)j[p] * j[q];
          AtB[p] += (double)j[p] * e;
        }
      }
      for (int k = 0; k < 36; ++k) a[k] = (float)AtA[k];
      for (int k = 0; k < 6; ++k) r[k] = (float)AtB[k];
    } else {  // general matrices
      for (int k = 0; k < 36; ++k) a[k] = nd(rng);
      for (int k = 0; k < 6; ++k) r[k] = nd(rng);
      if (kind == 6) a[(s / 8) % 36] = (s & 16) ? NAN : INFINITY;
      if (kind == 7) for (int k = 0; k < 6; ++k) a[k * 6 + 2] = 0.0f;  // a zero column
    }
  }
  float *dA, *db, *x0, *x1, *dout;
  int *ok0, *ok1;
  if (hipMalloc(&dA, A.size() * 4) || hipMalloc(&db, b.size() * 4) || hipMalloc(&x0, (size_t)n * 24) ||
      hipMalloc(&x1, (size_t)n * 24) || hipMalloc(&ok0, (size_t)n * 4) || hipMalloc(&ok1, (size_t)n * 4) ||
      hipMalloc(&dout, 16)) {
    std::printf("hip alloc error\n");
    return 2;
  }
  (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_ref, dim3(n / 64), dim3(64), 0, 0, dA, db, n, x0, ok0);
  hipLaunchKernelGGL(k_wave, dim3(n), dim3(64), 0, 0, dA, db, x1, ok1);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("hip error\n");
    return 2;
  }
  std::vector<uint32_t> h0((size_t)n * 6), h1((size_t)n * 6);
  std::vector<int> k0(n), k1(n);
  (void)hipMemcpy(h0.data(), x0, h0.size() * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(h1.data(), x1, h1.size() * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(k0.data(), ok0, (size_t)n * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(k1.data(), ok1, (size_t)n * 4, hipMemcpyDeviceToHost);
  long bad = 0, failed = 0, nan = 0;
  for (int s = 0; s < n; ++s) {
    // (a NaN solution matches a NaN: the sign of a generated NaN is not specified)
    bool same = k0[s] == k1[s];
    for (int k = 0; k < 6; ++k) {
      const uint32_t a = h0[(size_t)s * 6 + k], c = h1[(size_t)s * 6 + k];
      const bool an = (a & 0x7fffffffu) > 0x7f800000u, cn = (c & 0x7fffffffu) > 0x7f800000u;
      same = same && (a == c || (an && cn));
    }
    bad += same ? 0 : 1;
    failed += k0[s] ? 0 : 1;
    float f;
    std::memcpy(&f, &h0[(size_t)s * 6], 4);
    nan += std::isnan(f) ? 1 : 0;
    if (!same && bad <= 3)
      std::printf("system %d (kind %d): ok %d/%d x0 %08x/%08x\n", s, s % 8, k0[s], k1[s], h0[(size_t)s * 6],
                  h1[(size_t)s * 6]);
  }
  std::printf("qr_solve6_wave mismatches: %ld of %d systems (%ld singular exits, %ld NaN solutions)\n", bad, n,
              failed, nan);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int wave = 0; wave < 2; ++wave) {
    const int reps = 400;
    auto launch = [&](int r) {
      if (wave) hipLaunchKernelGGL(k_time<true>, dim3(1), dim3(64), 0, 0, dA, db, r, dout);
      else hipLaunchKernelGGL(k_time<false>, dim3(1), dim3(64), 0, 0, dA, db, r, dout);
    };
    launch(4);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    launch(reps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::printf("%s: %.3f us per solve\n", wave ? "qr_solve6_wave (one wave)" : "qr_solve (one lane)", 1e3 * ms / reps);
  }
  return bad ? 1 : 0;
}
