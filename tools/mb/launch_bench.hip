// Launch / sync cost on one stream (diagnostic): back-to-back trivial kernels (a one-workgroup
// kernel that returns at once, as a converged L-M launch does) and host round trips (async D2H of one
// int + hipStreamSynchronize).  hipcc --offload-arch=gfx950 -O2 tools/mb/launch_bench.hip -o /tmp/lb
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_noop(int* f) {
  if (f[0] == 12345) f[1] = 1;
}
__global__ void k_grid(int* f) {
  if (f[0] == 12345) f[blockIdx.x] = 1;
}

int main() {
  int *d = nullptr, *h = nullptr;
  hipMalloc(&d, 1 << 20);
  hipMemset(d, 0, 1 << 20);
  hipHostMalloc((void**)&h, 64, hipHostMallocDefault);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  auto now = [] { return std::chrono::steady_clock::now(); };
  for (int rep = 0; rep < 2; ++rep) {
    const int N = 2000;
    hipStreamSynchronize(s);
    auto a = now();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    const double t1 = std::chrono::duration<double, std::micro>(now() - a).count() / N;
    a = now();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_grid, dim3(256), dim3(256), 0, s, d);
    hipStreamSynchronize(s);
    const double t2 = std::chrono::duration<double, std::micro>(now() - a).count() / N;
    a = now();
    for (int i = 0; i < N / 10; ++i) {
      hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, s, d);
      hipMemcpyAsync(h, d, 4, hipMemcpyDeviceToHost, s);
      hipStreamSynchronize(s);
    }
    const double t3 = std::chrono::duration<double, std::micro>(now() - a).count() / (N / 10);
    if (rep) printf("noop 1 WG: %.2f us/launch; 256 WGs: %.2f us/launch; launch + D2H + sync: %.2f us\n", t1, t2, t3);
  }
  return 0;
}
