// Check of the DPP / permlane cross-lane forms (dev_common.hpp *_x) against the __shfl forms on
// random inputs, whole waves and 32-lane halves.  Built by loam_velodyne-1_amd/Makefile; run by
// tests/test_gpu_waveops.py on the GPU box.  Exit 0 when every result matches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#include "../../loam_velodyne-1_amd/csrc/dev_common.hpp"

using namespace loamdev;

constexpr int kOut = 10;  // per lane: min u64 x/ref, min f x/ref, scan x/ref, half scan x/ref, xor exchanges x/ref

__global__ void k_check(const uint64_t* keys, const float* fl, const int* iv, uint64_t* out) {
  const int w = blockIdx.x, lane = lane_id();
  const uint64_t k = keys[w * 64 + lane];
  const float f = fl[w * 64 + lane];
  const int v = iv[w * 64 + lane];
  uint64_t* o = out + ((size_t)w * 64 + lane) * kOut;
  o[0] = wave_min_u64_x(k);
  o[1] = wave_min_u64(k);
  o[2] = __float_as_uint(wave_min_f_x(f));
  o[3] = __float_as_uint(wave_min_f(f));
  o[4] = (uint32_t)wave_incl_scan_x(v);
  o[5] = (uint32_t)wave_incl_scan(v);
  // halves: 32-lane minimum of the keys and 32-lane inclusive scan
  o[6] = wave_min_u64_x<true>(k) ^ ((uint64_t)(uint32_t)wave_incl_scan_x<true>(v) << 1);
  uint64_t hm = k;
  for (int off = 16; off > 0; off >>= 1) {
    const uint64_t y = __shfl_xor(hm, off, 64);
    hm = y < hm ? y : hm;
  }
  int hs = v;
  for (int off = 1; off < 32; off <<= 1) {
    const int y = __shfl_up(hs, off, 32);
    if ((lane & 31) >= off) hs += y;
  }
  o[7] = hm ^ ((uint64_t)(uint32_t)hs << 1);
  // xor exchanges for every wave-uniform mask, folded into one word per lane
  uint64_t hx = 0, hr = 0;
  for (int m = 1; m < 64; m <<= 1) {
    hx = hx * 1000003u + (((uint64_t)xor_u32((uint32_t)(k >> 32), m) << 32) | xor_u32((uint32_t)k, m)) + (uint64_t)__float_as_uint((float)xor_f64((double)f, m));
    hr = hr * 1000003u + (((uint64_t)(uint32_t)__shfl_xor((int)(k >> 32), m, 64) << 32) | (uint32_t)__shfl_xor((int)(uint32_t)k, m, 64)) +
         (uint64_t)__float_as_uint((float)__shfl_xor((double)f, m, 64));
  }
  o[8] = hx;
  o[9] = hr;
}

int main() {
  constexpr int W = 4096;
  std::mt19937_64 rng(7);
  std::vector<uint64_t> keys(W * 64);
  std::vector<float> fl(W * 64);
  std::vector<int> iv(W * 64);
  for (int i = 0; i < W * 64; ++i) {
    const int mode = (i / 64) % 4;  // wave flavours: random, ties in the high word, sentinels, small
    const uint64_t r = rng();
    keys[i] = mode == 0 ? r : mode == 1 ? ((r & 7) << 32) | (r >> 40) : mode == 2 ? (r & 1 ? ~0ull : r) : r & 0xffff;
    fl[i] = mode == 2 && (r & 2) ? 3.4e38f : (float)((r >> 8) % 100000) * 0.001f - (mode == 3 ? 20.0f : 0.0f);
    iv[i] = (int)((r >> 20) % 1000) - (mode == 1 ? 500 : 0);
  }
  uint64_t *dk, *dout;
  float* df;
  int* di;
  (void)hipMalloc(&dk, keys.size() * 8);
  (void)hipMalloc(&df, fl.size() * 4);
  (void)hipMalloc(&di, iv.size() * 4);
  (void)hipMalloc(&dout, (size_t)W * 64 * kOut * 8);
  (void)hipMemcpy(dk, keys.data(), keys.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(df, fl.data(), fl.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(di, iv.data(), iv.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_check, dim3(W), dim3(64), 0, 0, dk, df, di, dout);
  std::vector<uint64_t> out((size_t)W * 64 * kOut);
  if (hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) {
    std::printf("hip error\n");
    return 2;
  }
  long bad[5] = {0, 0, 0, 0, 0};
  for (size_t i = 0; i < (size_t)W * 64; ++i)
    for (int c = 0; c < 5; ++c) bad[c] += out[i * kOut + 2 * c] != out[i * kOut + 2 * c + 1];
  std::printf("mismatches: min_u64 %ld, min_f %ld, scan %ld, half min+scan %ld, xor exchanges %ld over %d waves\n",
              bad[0], bad[1], bad[2], bad[3], bad[4], W);
  return (bad[0] || bad[1] || bad[2] || bad[3] || bad[4]) ? 1 : 0;
}
