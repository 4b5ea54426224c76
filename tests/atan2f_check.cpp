// Compares the engine's device atan2f (dev_common.hpp, compiled here for the host) with glibc's
// atan2f on sweep-like and random inputs; prints the number of bit mismatches.
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../loam_velodyne-1_amd/csrc/dev_common.hpp"
int main() {
  uint64_t s = 88172645463325252ull;
  long bad = 0, n = 0;
  auto bits = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
  for (long i = 0; i < 4000000; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    float a = (float)((int64_t)(s >> 11) % 200000) / 1000.0f;
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    float b = (float)((int64_t)(s >> 11) % 200000) / 1000.0f;
    if (s & 1) a = -a;
    if (s & 2) b = -b;
    if ((s & 12) == 12) a *= 1e-6f;
    ++n;
    if (bits(atan2f(a, b)) != bits(loamdev::atan2f_fdlibm(a, b))) ++bad;
  }
  std::printf("%ld %ld\n", n, bad);
  return 0;
}
