// Microbenchmark: where the ~4 us of the streaming odometry step goes (k_od_rows_small's last
// workgroup: the fp64 totals -> float normal equations, loamla::lm_step, the convergence test).
// Each piece runs `reps` times on one wave with a dependency between repetitions; us per call from
// HIP events.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../loam_velodyne-1_amd/csrc step_phases.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>

#include "dev_common.hpp"

#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(ck_)); return 1; } } while (0)

// MODE 0: lm_step (iter 1: the QR solve), 1: qr_solve alone on registers, 2: delta_r + delta_t,
// 3: totals (double, LDS) -> AtA / AtB (float, LDS) as od_step does, 4: 0 + 2 + 3 together
template <int MODE>
__global__ void k_piece(const double* tot_in, int reps, float* out) {
  __shared__ float ws[loamla::kLmWs];
  __shared__ int iws[12];
  __shared__ float sA[36], sB[6], X[6], P[36];
  __shared__ double tot[28];
  if (threadIdx.x < 28) tot[threadIdx.x] = tot_in[threadIdx.x];
  __syncthreads();
  if (threadIdx.x != 0) return;
  float acc = 0;
  for (int i = 0; i < 36; ++i) sA[i] = (float)tot[0];
  {
    int k = 0;
    for (int i = 0; i < 6; ++i)
      for (int jj = i; jj < 6; ++jj) { sA[i * 6 + jj] = sA[jj * 6 + i] = (float)tot[k]; ++k; }
    for (int i = 0; i < 6; ++i) sB[i] = (float)tot[21 + i];
  }
  for (int r = 0; r < reps; ++r) {
    if (MODE == 3 || MODE == 4) {
      tot[r % 27] += 1e-12 * acc;
      int k = 0;
      for (int i = 0; i < 6; ++i)
        for (int jj = i; jj < 6; ++jj) { sA[i * 6 + jj] = (float)tot[k]; sA[jj * 6 + i] = (float)tot[k]; ++k; }
      for (int i = 0; i < 6; ++i) sB[i] = (float)tot[21 + i];
    } else {
      sB[r % 6] += 1e-7f * acc;
    }
    if (MODE == 0 || MODE == 4) {
      int degen = 0;
      loamla::lm_step(sA, sB, 1, 10.0f, &degen, P, X, ws, iws);
      acc += X[0] + X[5];
    }
    if (MODE == 1) {
      float A[36], b[6], q[14], x[6];
      for (int i = 0; i < 36; ++i) A[i] = sA[i];
      for (int i = 0; i < 6; ++i) b[i] = sB[i];
      loamla::qr_solve(A, b, 6, 6, x, q);
      acc += x[0] + x[5];
    }
    if (MODE == 2 || MODE == 4) {
      float x[6];
      for (int i = 0; i < 6; ++i) x[i] = sB[i] * 1e-3f + acc * 1e-9f;
      const float dR = loamla::delta_r(x), dT = loamla::delta_t(x);
      acc += (dR < 0.1f && dT < 0.1f) ? 1e-3f : 2e-3f;
    }
    if (MODE == 3) acc += sA[7] + sB[3];
  }
  out[MODE] = acc;
}

template <int MODE>
int run(const double* d, float* o, const char* name) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_piece<MODE>, dim3(1), dim3(64), 0, 0, d, 4, o);
  CK(hipDeviceSynchronize());
  const int reps = 400;
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_piece<MODE>, dim3(1), dim3(64), 0, 0, d, reps, o);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-40s %.3f us per call\n", name, 1e3 * ms / reps);
  return 0;
}

int main() {
  std::mt19937 rng(7);
  std::normal_distribution<float> nd;
  double J[200 * 7], tot[28] = {};
  for (auto& v : J) v = nd(rng);
  for (int r = 0; r < 200; ++r) {
    int k = 0;
    for (int i = 0; i < 6; ++i)
      for (int j = i; j < 6; ++j) tot[k++] += J[r * 7 + i] * J[r * 7 + j];
    for (int i = 0; i < 6; ++i) tot[21 + i] += J[r * 7 + i] * 0.01 * J[r * 7 + 6];
    tot[27] += 1;
  }
  double* d;
  float* o;
  CK(hipMalloc(&d, sizeof(tot)));
  CK(hipMalloc(&o, 64));
  CK(hipMemcpy(d, tot, sizeof(tot), hipMemcpyHostToDevice));
  if (run<0>(d, o, "lm_step (iter 1)")) return 1;
  if (run<1>(d, o, "qr_solve 6x6 (registers)")) return 1;
  if (run<2>(d, o, "delta_r + delta_t")) return 1;
  if (run<3>(d, o, "totals -> AtA / AtB (LDS)")) return 1;
  if (run<4>(d, o, "conversion + lm_step + deltas")) return 1;
  return 0;
}
