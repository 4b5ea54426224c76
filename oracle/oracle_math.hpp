// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called from the product
// library (libloam_hip.so); only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use it.
//
// CPU restatements of the third-party numerics the reference calls but does not vendor
// (SURVEY.md §2 rows 13-15, appendix A2).  None of these libraries (PCL 1.7.1, OpenCV 2.4, tf of
// ROS Indigo) exists in this image and no reference test pins their results: PARITY UNPINNED at
// this boundary.  Each routine restates the published algorithm the call sites rely on:
//   KdTree      pcl::KdTreeFLANN<PointXYZI>::nearestKSearch — exact k-NN, squared L2 on xyz,
//               ascending; ties (equal float distance) broken by lower point index.
//               call sites: src/laserOdometry.cpp:478,590  src/laserMapping.cpp:717,824
//   voxel_grid  pcl::VoxelGrid<PointXYZI>::filter (downsample_all_data_ = true) — float leaf
//               inverse, bbox, floor keys, sort by linear voxel index (stable: equal keys keep
//               input order), float centroid of x,y,z,intensity, "leaf too small" pass-through.
//               call sites: src/scanRegistration.cpp:575-579  src/laserMapping.cpp:694-700,1022-1027
//   gemm_d      cv::Mat * cv::Mat for CV_32F — products and sums in double, one rounding to float
//   qr_solve    cv::solve(..., DECOMP_QR) — float Householder QR + back substitution (m >= n)
//   jacobi      cv::eigen on symmetric float — cyclic-max-pivot Jacobi, eigenvalues descending,
//               eigenvectors as rows
//   lu_inv      cv::Mat::inv() (DECOMP_LU) — float Gaussian elimination, partial pivoting
//   tf_*        tf::Quaternion::setRPY / tf::Matrix3x3::getRPY in double (message conventions)
#ifndef LOAM_ORACLE_MATH_HPP
#define LOAM_ORACLE_MATH_HPP

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

namespace oracle {

struct P { float x, y, z, intensity; };

// ---------------------------------------------------------------- kd-tree (exact k-NN)
class KdTree {
 public:
  void build(const std::vector<P>& pts) {
    pts_ = &pts;
    nodes_.clear();
    idx_.resize(pts.size());
    for (size_t i = 0; i < pts.size(); ++i) idx_[i] = (int)i;
    if (!pts.empty()) build_rec(0, (int)pts.size());
  }
  bool empty() const { return pts_ == nullptr || pts_->empty(); }
  // k nearest (ascending by (distance, index)); returns the number found (< k if cloud small)
  int knn(float qx, float qy, float qz, int k, int* out_idx, float* out_d) const {
    nfound_ = 0;
    k_ = k;
    bi_ = out_idx;
    bd_ = out_d;
    q_[0] = qx; q_[1] = qy; q_[2] = qz;
    if (!empty()) search(0);
    return nfound_;
  }

 private:
  struct Node { float lo[3], hi[3]; int begin, end, left, right; };
  static float coord(const P& p, int d) { return d == 0 ? p.x : (d == 1 ? p.y : p.z); }
  int build_rec(int b, int e) {
    Node n;
    n.begin = b; n.end = e; n.left = n.right = -1;
    for (int d = 0; d < 3; ++d) { n.lo[d] = FLT_MAX; n.hi[d] = -FLT_MAX; }
    for (int i = b; i < e; ++i)
      for (int d = 0; d < 3; ++d) {
        float c = coord((*pts_)[idx_[i]], d);
        n.lo[d] = std::min(n.lo[d], c);
        n.hi[d] = std::max(n.hi[d], c);
      }
    int id = (int)nodes_.size();
    nodes_.push_back(n);
    if (e - b > kLeaf) {
      int dim = 0;
      float span = n.hi[0] - n.lo[0];
      for (int d = 1; d < 3; ++d)
        if (n.hi[d] - n.lo[d] > span) { span = n.hi[d] - n.lo[d]; dim = d; }
      int m = b + (e - b) / 2;
      const std::vector<P>& pts = *pts_;
      std::nth_element(idx_.begin() + b, idx_.begin() + m, idx_.begin() + e,
                       [&](int a, int c) {
                         float ca = coord(pts[a], dim), cc = coord(pts[c], dim);
                         return ca < cc || (ca == cc && a < c);
                       });
      int l = build_rec(b, m);
      int r = build_rec(m, e);
      nodes_[id].left = l;
      nodes_[id].right = r;
    }
    return id;
  }
  // lower bound of the float squared distance from q to any point in the box (never above the
  // float distance of a point inside it: rounding is monotone)
  float box_lb(const Node& n) const {
    float s = 0.0f;
    for (int d = 0; d < 3; ++d) {
      float g = 0.0f;
      if (q_[d] < n.lo[d]) g = n.lo[d] - q_[d];
      else if (q_[d] > n.hi[d]) g = q_[d] - n.hi[d];
      s = s + g * g;
    }
    return s;
  }
  void offer(int i, float d) const {
    // insert (d, i) into the ascending top-k list
    if (nfound_ == k_) {
      if (d > bd_[k_ - 1] || (d == bd_[k_ - 1] && i > bi_[k_ - 1])) return;
      --nfound_;
    }
    int j = nfound_;
    while (j > 0 && (bd_[j - 1] > d || (bd_[j - 1] == d && bi_[j - 1] > i))) {
      bd_[j] = bd_[j - 1];
      bi_[j] = bi_[j - 1];
      --j;
    }
    bd_[j] = d;
    bi_[j] = i;
    ++nfound_;
  }
  void search(int id) const {
    const Node& n = nodes_[id];
    if (nfound_ == k_ && box_lb(n) > bd_[k_ - 1]) return;
    if (n.left < 0) {
      const std::vector<P>& pts = *pts_;
      for (int i = n.begin; i < n.end; ++i) {
        const P& p = pts[idx_[i]];
        float dx = p.x - q_[0], dy = p.y - q_[1], dz = p.z - q_[2];
        offer(idx_[i], dx * dx + dy * dy + dz * dz);
      }
      return;
    }
    float bl = box_lb(nodes_[n.left]), br = box_lb(nodes_[n.right]);
    if (bl <= br) { search(n.left); search(n.right); }
    else { search(n.right); search(n.left); }
  }
  static const int kLeaf = 15;  // FLANN KDTreeSingleIndex leaf size used by KdTreeFLANN
  const std::vector<P>* pts_ = nullptr;
  std::vector<Node> nodes_;
  std::vector<int> idx_;
  mutable float q_[3];
  mutable int k_ = 0, nfound_ = 0;
  mutable int* bi_ = nullptr;
  mutable float* bd_ = nullptr;
};

// ---------------------------------------------------------------- PCL VoxelGrid
// PCL's overflow test: (int64)((max-min)*inv)+1 per axis, product > INT_MAX -> output = input.
// PCL's own product (and its int conversion of the scaled bbox) is undefined for spans beyond
// int range; those cases are defined here as "too small" too (same rule as the engine).
inline bool vg_leaf_too_small(const float* mn, const float* mx, float inv) {
  int64_t e[3];
  for (int d = 0; d < 3; ++d) {
    const float sp = (mx[d] - mn[d]) * inv, lo = mn[d] * inv, hi = mx[d] * inv;
    if (!(sp < 2147483648.0f) || !(lo >= -2147483648.0f) || !(hi < 2147483648.0f)) return true;
    e[d] = (int64_t)sp + 1;
  }
  const int64_t xy = e[0] * e[1];
  return xy > (int64_t)INT32_MAX || xy * e[2] > (int64_t)INT32_MAX;
}

inline void voxel_grid(const std::vector<P>& in, float leaf, std::vector<P>& out) {
  out.clear();
  if (in.empty()) return;
  const float inv = 1.0f / leaf;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (const P& p : in) {
    const float c[3] = {p.x, p.y, p.z};
    for (int d = 0; d < 3; ++d) { mn[d] = std::min(mn[d], c[d]); mx[d] = std::max(mx[d], c[d]); }
  }
  if (vg_leaf_too_small(mn, mx, inv)) {  // "Leaf size is too small": output = input
    out = in;
    return;
  }
  int minb[3], maxb[3];
  for (int d = 0; d < 3; ++d) {
    minb[d] = (int)std::floor(mn[d] * inv);
    maxb[d] = (int)std::floor(mx[d] * inv);
  }
  const int divx = maxb[0] - minb[0] + 1, divy = maxb[1] - minb[1] + 1;
  const int mul1 = divx, mul2 = divx * divy;
  std::vector<std::pair<uint32_t, uint32_t>> keys(in.size());
  for (size_t i = 0; i < in.size(); ++i) {
    const P& p = in[i];
    int i0 = (int)(std::floor(p.x * inv) - (float)minb[0]);
    int i1 = (int)(std::floor(p.y * inv) - (float)minb[1]);
    int i2 = (int)(std::floor(p.z * inv) - (float)minb[2]);
    keys[i] = std::make_pair((uint32_t)(i0 + i1 * mul1 + i2 * mul2), (uint32_t)i);
  }
  std::sort(keys.begin(), keys.end());   // (voxel index, input position): stable order per voxel
  size_t b = 0;
  while (b < keys.size()) {
    size_t e = b + 1;
    while (e < keys.size() && keys[e].first == keys[b].first) ++e;
    float s[4] = {0, 0, 0, 0};
    for (size_t k = b; k < e; ++k) {
      const P& p = in[keys[k].second];
      s[0] += p.x; s[1] += p.y; s[2] += p.z; s[3] += p.intensity;
    }
    const float cnt = (float)(e - b);
    out.push_back(P{s[0] / cnt, s[1] / cnt, s[2] / cnt, s[3] / cnt});
    b = e;
  }
}

// ---------------------------------------------------------------- OpenCV float gemm (double acc)
// C[m x n] = A[m x k] * B[k x n], row-major
inline void gemm_d(const float* A, const float* B, int m, int k, int n, float* C) {
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int l = 0; l < k; ++l) s += (double)A[i * k + l] * (double)B[l * n + j];
      C[i * n + j] = (float)s;
    }
}

// ---------------------------------------------------------------- OpenCV DECOMP_QR (float)
// Solves A x = b in the least-squares sense for an m x n (m >= n) float A; A, b are copied.
// Returns false when a diagonal of R is below 10*FLT_EPSILON (cv::solve then outputs zeros).
inline bool qr_solve(const float* Ain, const float* bin, int m, int n, float* x) {
  std::vector<float> A(Ain, Ain + m * n), b(bin, bin + m), v(m), h(n);
  const float eps = FLT_EPSILON * 10;
  for (int l = 0; l < n; ++l) {
    const int len = m - l;
    float nrm = 0.0f;
    for (int i = 0; i < len; ++i) { v[i] = A[(l + i) * n + l]; nrm += v[i] * v[i]; }
    const float v0 = v[0];
    v[0] = v[0] + (v[0] >= 0.0f ? 1.0f : -1.0f) * std::sqrt(nrm);
    nrm = std::sqrt(nrm + v[0] * v[0] - v0 * v0);
    for (int i = 0; i < len; ++i) v[i] /= nrm;
    for (int j = l; j < n; ++j) {
      float dot = 0.0f;
      for (int i = l; i < m; ++i) dot += v[i - l] * A[i * n + j];
      for (int i = l; i < m; ++i) A[i * n + j] -= 2 * v[i - l] * dot;
    }
    h[l] = v[0] * v[0];
    for (int i = 1; i < len; ++i) A[(l + i) * n + l] = v[i] / v[0];
  }
  for (int l = 0; l < n; ++l) {
    v[0] = 1.0f;
    for (int j = 1; j < m - l; ++j) v[j] = A[(j + l) * n + l];
    float dot = 0.0f;
    for (int i = l; i < m; ++i) dot += v[i - l] * b[i];
    for (int i = l; i < m; ++i) b[i] -= 2 * v[i - l] * dot * h[l];
  }
  for (int i = n - 1; i >= 0; --i) {
    for (int j = n - 1; j > i; --j) b[i] -= b[j] * A[i * n + j];
    if (std::fabs(A[i * n + i]) < eps) {
      for (int q = 0; q < n; ++q) x[q] = 0.0f;
      return false;
    }
    b[i] /= A[i * n + i];
  }
  for (int i = 0; i < n; ++i) x[i] = b[i];
  return true;
}

// ---------------------------------------------------------------- OpenCV eigen (Jacobi, float)
inline float hypot_cv(float a, float b) {
  a = std::fabs(a);
  b = std::fabs(b);
  if (a > b) { b /= a; return a * std::sqrt(1 + b * b); }
  if (b > 0) { a /= b; return b * std::sqrt(1 + a * a); }
  return 0;
}

// A (n x n symmetric, destroyed copy) -> W eigenvalues descending, V eigenvectors as rows
inline void jacobi(const float* Ain, int n, float* W, float* V) {
  std::vector<float> A(Ain, Ain + n * n);
  std::vector<int> indR(n, 0), indC(n, 0);
  const float eps = FLT_EPSILON;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0f : 0.0f;
  auto rowmax = [&](int k) {  // column of the largest |A[k][m]|, m > k
    int m = k + 1;
    float mv = std::fabs(A[k * n + m]);
    for (int i = k + 2; i < n; ++i) {
      float val = std::fabs(A[k * n + i]);
      if (mv < val) { mv = val; m = i; }
    }
    indR[k] = m;
  };
  auto colmax = [&](int k) {  // row of the largest |A[m][k]|, m < k
    int m = 0;
    float mv = std::fabs(A[k]);
    for (int i = 1; i < k; ++i) {
      float val = std::fabs(A[i * n + k]);
      if (mv < val) { mv = val; m = i; }
    }
    indC[k] = m;
  };
  for (int k = 0; k < n; ++k) {
    W[k] = A[k * n + k];
    if (k < n - 1) rowmax(k);
    if (k > 0) colmax(k);
  }
  if (n > 1) {
    for (int iters = 0; iters < n * n * 30; ++iters) {
      int k = 0;
      float mv = std::fabs(A[indR[0]]);
      for (int i = 1; i < n - 1; ++i) {
        float val = std::fabs(A[i * n + indR[i]]);
        if (mv < val) { mv = val; k = i; }
      }
      int l = indR[k];
      for (int i = 1; i < n; ++i) {
        float val = std::fabs(A[indC[i] * n + i]);
        if (mv < val) { mv = val; k = indC[i]; l = i; }
      }
      float p = A[k * n + l];
      if (std::fabs(p) <= eps) break;
      float y = (float)((W[l] - W[k]) * 0.5);
      float t = std::fabs(y) + hypot_cv(p, y);
      float s = hypot_cv(p, t);
      float c = t / s;
      s = p / s;
      t = (p / t) * p;
      if (y < 0) { s = -s; t = -t; }
      A[k * n + l] = 0;
      W[k] -= t;
      W[l] += t;
      auto rot = [&](float& v0, float& v1) {
        float a0 = v0, b0 = v1;
        v0 = a0 * c - b0 * s;
        v1 = a0 * s + b0 * c;
      };
      for (int i = 0; i < k; ++i) rot(A[i * n + k], A[i * n + l]);
      for (int i = k + 1; i < l; ++i) rot(A[k * n + i], A[i * n + l]);
      for (int i = l + 1; i < n; ++i) rot(A[k * n + i], A[l * n + i]);
      for (int i = 0; i < n; ++i) rot(V[k * n + i], V[l * n + i]);
      for (int j = 0; j < 2; ++j) {
        int idx = j == 0 ? k : l;
        if (idx < n - 1) rowmax(idx);
        if (idx > 0) colmax(idx);
      }
    }
  }
  for (int k = 0; k < n - 1; ++k) {  // selection sort, descending
    int m = k;
    for (int i = k + 1; i < n; ++i)
      if (W[m] < W[i]) m = i;
    if (k != m) {
      std::swap(W[m], W[k]);
      for (int i = 0; i < n; ++i) std::swap(V[m * n + i], V[k * n + i]);
    }
  }
}

// ---------------------------------------------------------------- OpenCV inv (LU, float)
inline bool lu_inv(const float* Ain, int n, float* Inv) {
  std::vector<float> A(Ain, Ain + n * n), b(n * n, 0.0f);
  for (int i = 0; i < n; ++i) b[i * n + i] = 1.0f;
  const float eps = FLT_EPSILON * 10;
  for (int i = 0; i < n; ++i) {
    int k = i;
    for (int j = i + 1; j < n; ++j)
      if (std::fabs(A[j * n + i]) > std::fabs(A[k * n + i])) k = j;
    if (std::fabs(A[k * n + i]) < eps) {
      for (int q = 0; q < n * n; ++q) Inv[q] = 0.0f;
      return false;
    }
    if (k != i) {
      for (int j = i; j < n; ++j) std::swap(A[i * n + j], A[k * n + j]);
      for (int j = 0; j < n; ++j) std::swap(b[i * n + j], b[k * n + j]);
    }
    float d = -1 / A[i * n + i];
    for (int j = i + 1; j < n; ++j) {
      float alpha = A[j * n + i] * d;
      for (int q = i + 1; q < n; ++q) A[j * n + q] += alpha * A[i * n + q];
      for (int q = 0; q < n; ++q) b[j * n + q] += alpha * b[i * n + q];
    }
  }
  for (int i = n - 1; i >= 0; --i)
    for (int j = 0; j < n; ++j) {
      float s = b[i * n + j];
      for (int q = i + 1; q < n; ++q) s -= A[i * n + q] * b[q * n + j];
      b[i * n + j] = s / A[i * n + i];
    }
  for (int q = 0; q < n * n; ++q) Inv[q] = b[q];
  return true;
}

// ---------------------------------------------------------------- tf quaternion <-> RPY (double)
struct Quat { double x, y, z, w; };
inline Quat tf_from_rpy(double roll, double pitch, double yaw) {
  double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
  double cy = std::cos(hy), sy = std::sin(hy), cp = std::cos(hp), sp = std::sin(hp);
  double cr = std::cos(hr), sr = std::sin(hr);
  return Quat{sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
              cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy};
}
inline void tf_get_rpy(const Quat& q, double& roll, double& pitch, double& yaw) {
  double d = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
  double s = 2.0 / d;
  double xs = q.x * s, ys = q.y * s, zs = q.z * s;
  double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
  double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
  double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
  double m00 = 1.0 - (yy + zz), m02 = xz + wy;
  double m10 = xy + wz;
  double m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
  if (std::fabs(m20) >= 1) {
    yaw = 0;
    double delta = std::atan2(m00, m02);
    if (m20 > 0) { pitch = M_PI / 2.0; roll = pitch + delta; }
    else { pitch = -M_PI / 2.0; roll = -pitch + delta; }
  } else {
    pitch = -std::asin(m20);
    roll = std::atan2(m21 / std::cos(pitch), m22 / std::cos(pitch));
    yaw = std::atan2(m10 / std::cos(pitch), m00 / std::cos(pitch));
  }
}

}  // namespace oracle
#endif
