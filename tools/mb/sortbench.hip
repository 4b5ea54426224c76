// Microbenchmark: hipCUB segmented radix sort (as vg_run uses it) vs one global radix sort over
// (segment, voxel) composite keys, on VoxelGrid-shaped data.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
#include <random>
#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(ck_)); return 1; } } while (0)
int run(int nseg, int segn, int gap, int keybits, int segn2 = -1) {
  if (segn2 < 0) segn2 = segn;
  const int total = nseg * (segn + gap);
  std::vector<int> b(nseg), e(nseg);
  std::vector<uint32_t> k(total), v(total);
  std::vector<uint64_t> ck(nseg * segn);
  std::vector<uint32_t> cv(nseg * segn);
  std::mt19937 rng(1);
  for (int s = 0; s < nseg; ++s) {
    b[s] = s * (segn + gap); e[s] = b[s] + ((s & 1) ? segn2 : segn);
    for (int i = 0; i < e[s] - b[s]; ++i) {
      k[b[s] + i] = rng() & ((1u << keybits) - 1);
      v[b[s] + i] = b[s] + i;
      ck[s * segn + i] = ((uint64_t)s << 32) | k[b[s] + i];
      cv[s * segn + i] = b[s] + i;
    }
  }
  uint32_t *dk, *dk2, *dv, *dv2; int *db, *de; uint64_t *dck, *dck2; uint32_t *dcv, *dcv2;
  CK(hipMalloc(&dk, total * 4)); CK(hipMalloc(&dk2, total * 4)); CK(hipMalloc(&dv, total * 4)); CK(hipMalloc(&dv2, total * 4));
  CK(hipMalloc(&db, nseg * 4)); CK(hipMalloc(&de, nseg * 4));
  const int nc = nseg * segn;
  CK(hipMalloc(&dck, nc * 8)); CK(hipMalloc(&dck2, nc * 8)); CK(hipMalloc(&dcv, nc * 4)); CK(hipMalloc(&dcv2, nc * 4));
  CK(hipMemcpy(dk, k.data(), total * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(dv, v.data(), total * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, b.data(), nseg * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(de, e.data(), nseg * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dck, ck.data(), nc * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dcv, cv.data(), nc * 4, hipMemcpyHostToDevice));
  size_t t1 = 0, t2 = 0;
  hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, t1, dk, dk2, dv, dv2, total, nseg, db, de, 0, 32);
  int segbits = 0; while ((1 << segbits) < nseg) ++segbits;
  hipcub::DeviceRadixSort::SortPairs(nullptr, t2, dck, dck2, dcv, dcv2, nc, 0, 32 + segbits);
  void* tmp; CK(hipMalloc(&tmp, t1 > t2 ? t1 : t2));
  hipEvent_t a, c; hipEventCreate(&a); hipEventCreate(&c);
  float ms1 = 0, ms2 = 0, ms3 = 0;
  for (int it = 0; it < 6; ++it) {
    size_t tt = t1;
    hipEventRecord(a);
    hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tt, dk, dk2, dv, dv2, total, nseg, db, de, 0, 32);
    hipEventRecord(c); hipEventSynchronize(c);
    float m; hipEventElapsedTime(&m, a, c); if (it) ms1 += m / 5;
    tt = t2;
    hipEventRecord(a);
    hipcub::DeviceRadixSort::SortPairs(tmp, tt, dck, dck2, dcv, dcv2, nc, 0, 32 + segbits);
    hipEventRecord(c); hipEventSynchronize(c);
    hipEventElapsedTime(&m, a, c); if (it) ms2 += m / 5;
    tt = t2;
    hipEventRecord(a);
    hipcub::DeviceRadixSort::SortPairs(tmp, tt, dck, dck2, dcv, dcv2, nc, 0, keybits + segbits > 32 ? 64 : 32);
    hipEventRecord(c); hipEventSynchronize(c);
    hipEventElapsedTime(&m, a, c); if (it) ms3 += m / 5;
  }
  printf("nseg %d segn %d keybits %d: segmented %.3f ms, global(%d bits) %.3f ms, global(64/32 bits) %.3f ms\n", nseg, segn, keybits, ms1, 32 + segbits, ms2, ms3);
  return 0;
}
int main() {
  run(2048, 4500, 10000, 26, 1000);
  run(2048, 4500, 0, 26, 1000);
  run(2048, 2500, 500, 26);
  run(2048, 5000, 0, 26, 0);
  return 0;
}
