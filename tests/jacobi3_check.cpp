// Host check (tests/test_jacobi3.py): loamla::jacobi3_reg against loamla::jacobi<3> (dev_common.hpp
// compiled for the host), bit for bit, on random symmetric 3x3 matrices shaped like the mapping's
// corner covariances (a dominant direction, near-ties, exact zeros, repeated eigenvalues).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../loam_velodyne-1_amd/csrc/dev_common.hpp"

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937 rng(12345);
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  long bad = 0;
  for (long it = 0; it < n; ++it) {
    float A[9];
    const int kind = (int)(it % 5);
    float pts[5][3];
    for (int k = 0; k < 5; ++k)
      for (int d = 0; d < 3; ++d) pts[k][d] = u(rng) * (kind == 0 && d > 0 ? 0.01f : 1.0f);
    if (kind == 1)  // collinear points (two zero eigenvalues)
      for (int k = 0; k < 5; ++k) { pts[k][1] = pts[k][0] * 0.5f; pts[k][2] = pts[k][0] * -2.0f; }
    if (kind == 2)  // a diagonal matrix with ties
      for (int k = 0; k < 5; ++k) { pts[k][1] = (k & 1) ? 0.5f : -0.5f; pts[k][2] = (k & 1) ? -0.5f : 0.5f; }
    float c[3] = {0, 0, 0};
    for (int k = 0; k < 5; ++k) for (int d = 0; d < 3; ++d) c[d] += pts[k][d];
    for (int d = 0; d < 3; ++d) c[d] /= 5;
    float a[6] = {0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 5; ++k) {
      const float x = pts[k][0] - c[0], y = pts[k][1] - c[1], z = pts[k][2] - c[2];
      a[0] += x * x; a[1] += x * y; a[2] += x * z; a[3] += y * y; a[4] += y * z; a[5] += z * z;
    }
    for (int d = 0; d < 6; ++d) a[d] /= 5;
    if (kind == 3) { a[1] = 0; a[2] = 0; a[4] = 0; }  // already diagonal
    if (kind == 4 && (it & 8)) { a[0] = a[3]; a[5] = a[3]; }  // equal diagonal
    A[0] = a[0]; A[1] = a[1]; A[2] = a[2]; A[3] = a[1]; A[4] = a[3]; A[5] = a[4]; A[6] = a[2]; A[7] = a[4]; A[8] = a[5];
    float A1[9], W1[3], V1[9], W2[3], V2[9];
    int iws[6];
    memcpy(A1, A, sizeof(A));
    loamla::jacobi<3>(A1, W1, V1, iws);
    loamla::jacobi3_reg(A, W2, V2);
    if (memcmp(W1, W2, sizeof(W1)) || memcmp(V1, V2, sizeof(V1))) ++bad;
  }
  printf("%ld %ld\n", n, bad);
  return 0;
}
