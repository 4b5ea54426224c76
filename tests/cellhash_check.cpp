// The map search's exactness rests on cell_hash (dev_common.hpp, compiled here for the host) never
// sending two of the 27 cells around any cell to one bucket of a table of >= 64 buckets: the 5-NN
// list then meets every map point at most once and needs no duplicate test (mp.hip knn5_flat).
// Checks random cells over +-2^20 and every table size 2^6 .. 2^20; prints "<checked> <collisions>".
#include <cstdint>
#include <cstdio>
#include "../loam_velodyne-1_amd/csrc/dev_common.hpp"
int main() {
  uint64_t s = 0x9e3779b97f4a7c15ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (int)(s % 2097152) - 1048576; };
  long checked = 0, coll = 0;
  for (int trial = 0; trial < 200000; ++trial) {
    const int cx = rnd(), cy = rnd() % 4096, cz = rnd() % 512;
    for (int lg = 6; lg <= 20; ++lg) {
      const uint32_t T = 1u << lg;
      uint32_t h[27];
      for (int c = 0; c < 27; ++c)
        h[c] = loamdev::cell_hash(cx + c % 3 - 1, cy + (c / 3) % 3 - 1, cz + c / 9 - 1) & (T - 1);
      for (int a = 0; a < 27; ++a)
        for (int b = a + 1; b < 27; ++b) coll += h[a] == h[b];
      ++checked;
    }
  }
  std::printf("%ld %ld\n", checked, coll);
  return 0;
}
