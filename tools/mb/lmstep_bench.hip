// Microbenchmark: the device cost of the 6x6 L-M step (loamla::lm_step on one lane: QR solve every
// iteration, pivoted Jacobi + LU + projection at iteration 0) and of a bare dependent launch, to
// size the single-stream latency budget.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../loam_velodyne-1_amd/csrc lmstep_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>

#include "dev_common.hpp"

#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(ck_)); return 1; } } while (0)

__global__ void k_step(const float* AtA, const float* AtB, int iter, int reps, float* out) {
  __shared__ float ws[loamla::kLmWs];
  __shared__ int iws[12];
  __shared__ float sA[36], sB[6], X[6], P[36];
  if (threadIdx.x == 0) {
    for (int i = 0; i < 36; ++i) sA[i] = AtA[i];
    for (int i = 0; i < 6; ++i) sB[i] = AtB[i];
    float acc = 0;
    for (int r = 0; r < reps; ++r) {
      int degen = 0;
      sB[r % 6] += 1e-7f * acc;  // keep the calls dependent
      loamla::lm_step(sA, sB, iter, 10.0f, &degen, P, X, ws, iws);
      acc += X[0] + X[5] + (float)degen;
    }
    out[0] = acc;
  }
}

__global__ void k_empty(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] += 1.0f;
}

int main() {
  std::mt19937 rng(7);
  std::normal_distribution<float> nd;
  float J[60 * 6], AtA[36] = {}, AtB[6] = {};
  for (auto& v : J) v = nd(rng);
  for (int r = 0; r < 60; ++r)
    for (int i = 0; i < 6; ++i) {
      for (int j = 0; j < 6; ++j) AtA[i * 6 + j] += J[r * 6 + i] * J[r * 6 + j];
      AtB[i] += J[r * 6 + i] * 0.01f;
    }
  float *dA, *dB, *dO;
  CK(hipMalloc(&dA, sizeof(AtA)));
  CK(hipMalloc(&dB, sizeof(AtB)));
  CK(hipMalloc(&dO, 16));
  CK(hipMemcpy(dA, AtA, sizeof(AtA), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, AtB, sizeof(AtB), hipMemcpyHostToDevice));
  CK(hipMemset(dO, 0, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int iter = 0; iter < 2; ++iter) {
    const int reps = 200;
    hipLaunchKernelGGL(k_step, dim3(1), dim3(64), 0, 0, dA, dB, iter, 4, dO);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_step, dim3(1), dim3(64), 0, 0, dA, dB, iter, reps, dO);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("lm_step iter=%d: %.2f us per call (one lane)\n", iter, 1e3 * ms / reps);
  }
  // dependent launches back to back
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, dO);
  CK(hipDeviceSynchronize());
  const int nl = 1000;
  CK(hipEventRecord(e0));
  for (int i = 0; i < nl; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, dO);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("empty dependent launch: %.2f us each\n", 1e3 * ms / nl);
  return 0;
}
