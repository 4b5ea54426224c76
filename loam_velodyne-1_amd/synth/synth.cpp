// Deterministic synthetic lidar sweep generator (test / bench input only).
//
// The reference is validated on recorded bags (nsh_indoor_outdoor.bag, laboshinl's VLP-16 bag,
// /root/reference/README.md:22-35) that are not available offline, so every config in
// BASELINE.json runs on sweeps produced here.  The generator models what the reference's
// scanRegistration expects from the velodyne driver (src/scanRegistration.cpp:225-351):
//   * points in the instantaneous sensor frame (x forward, y left, z up), one per laser firing,
//     emitted azimuth-major in laser firing order;
//   * clockwise rotation: velodyne-frame atan2(y, x) decreases with time, so the reference's
//     ori = -atan2(y, x) increases through the sweep (src/scanRegistration.cpp:262);
//   * motion distortion: each firing sees the world from the pose at its own time;
//   * misses and returns beyond max range are dropped (no NaN), Gaussian range noise.
// All arithmetic is double precision with explicitly seeded splitmix64 streams, so the output is
// identical wherever glibc's libm is identical (this image, here and on the GPU box).
#include "synth.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Box { double lo[3], hi[3]; };
struct Plane { double n[3], d; };

struct Scene {
  std::vector<Box> boxes;
  std::vector<Plane> planes;
};

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  double uni(double a, double b) { return a + (b - a) * uni(); }
  double gauss() {
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
};

void add_box(Scene& s, double x0, double y0, double z0, double x1, double y1, double z1) {
  Box b;
  b.lo[0] = x0 < x1 ? x0 : x1; b.hi[0] = x0 < x1 ? x1 : x0;
  b.lo[1] = y0 < y1 ? y0 : y1; b.hi[1] = y0 < y1 ? y1 : y0;
  b.lo[2] = z0 < z1 ? z0 : z1; b.hi[2] = z0 < z1 ? z1 : z0;
  s.boxes.push_back(b);
}

// Outer shell: makes every laser of every ring return something within max range, so no ring is
// ever empty (an empty ring triggers reference quirk Q5).
void add_enclosure(Scene& s, double half, double zlo, double zhi) {
  const double t = 0.5;
  add_box(s, -half - t, -half - t, zlo - t, half + t, -half, zhi + t);
  add_box(s, -half - t, half, zlo - t, half + t, half + t, zhi + t);
  add_box(s, -half - t, -half, zlo - t, -half, half, zhi + t);
  add_box(s, half, -half, zlo - t, half + t, half, zhi + t);
  add_box(s, -half, -half, zhi, half, half, zhi + t);      // ceiling
  add_box(s, -half, -half, zlo - t, half, half, zlo);      // floor slab
}

// "Indoor-outdoor" scene of SURVEY.md §8(d) configs 1-3: ground at z=-1.5, a 20x30x4 m room with
// door gaps, 8 pillars, boxes, inside a large enclosure.
void build_indoor(Scene& s, uint64_t seed) {
  Rng r(seed ^ 0x1D00ull);
  add_enclosure(s, 45.0, -1.5, 18.0);
  const double g = -1.5, h = 4.0 + g, th = 0.2;
  // room walls x in [-10,10], y in [-15,15], with door gaps
  add_box(s, -10, -15, g, -1.0, -15 + th, h);
  add_box(s, 1.0, -15, g, 10, -15 + th, h);
  add_box(s, -10, 15 - th, g, 10, 15, h);
  add_box(s, -10, -15, g, -10 + th, -4.0, h);
  add_box(s, -10, -2.0, g, -10 + th, 15, h);
  add_box(s, 10 - th, -15, g, 10, 6.0, h);
  add_box(s, 10 - th, 8.0, g, 10, 15, h);
  // 8 pillars (vertical edges)
  const double px[8] = {-6, 6, -6, 6, -3, 3, -7.5, 7.5};
  const double py[8] = {-9, -9, 9, 9, 0.5, -0.5, 1, -1};
  for (int i = 0; i < 8; ++i)
    add_box(s, px[i] - 0.2, py[i] - 0.2, g, px[i] + 0.2, py[i] + 0.2, g + 5.0);
  // boxes of random size, kept off the circular driving lane of the config-3 loop (radius 6 m
  // around the origin, synthgen.loop_pose): a box whose footprint reaches radii 3.5 .. 8.5 m is
  // re-drawn (bounded, deterministic)
  for (int i = 0; i < 10; ++i) {
    double sx = r.uni(0.4, 1.5), sy = r.uni(0.4, 1.5), sz = r.uni(0.5, 2.0);
    double cx = 0, cy = 0;
    for (int tries = 0; tries < 64; ++tries) {
      cx = r.uni(-8.5, 8.5);
      cy = r.uni(-13.5, 13.5);
      const double dmin = std::hypot(std::max(std::fabs(cx) - sx, 0.0), std::max(std::fabs(cy) - sy, 0.0));
      const double dmax = std::hypot(std::fabs(cx) + sx, std::fabs(cy) + sy);
      if (dmin >= 8.5 || dmax <= 3.5) break;
    }
    add_box(s, cx - sx, cy - sy, g, cx + sx, cy + sy, g + sz);
  }
  // outdoor structures beyond the room
  for (int i = 0; i < 12; ++i) {
    double a = r.uni(0, 2 * M_PI), d = r.uni(20, 38);
    double cx = d * std::cos(a), cy = d * std::sin(a);
    double sx = r.uni(1, 4), sy = r.uni(1, 4), sz = r.uni(2, 12);
    add_box(s, cx - sx, cy - sy, g, cx + sx, cy + sy, g + sz);
  }
}

// Random planes + edges scene of SURVEY.md §8(d) config 4 (seeds 1000..2023).
void build_random(Scene& s, uint64_t seed) {
  Rng r(seed ^ 0x5EEDull);
  add_enclosure(s, 60.0, -2.0, 25.0);
  int np = 6 + (int)(r.next() % 7);
  for (int i = 0; i < np; ++i) {
    double z = r.uni(-1, 1), a = r.uni(0, 2 * M_PI), rr = std::sqrt(1 - z * z);
    Plane p;
    p.n[0] = rr * std::cos(a); p.n[1] = rr * std::sin(a); p.n[2] = z;
    p.d = r.uni(3, 30);
    s.planes.push_back(p);
  }
  Plane ground; ground.n[0] = 0; ground.n[1] = 0; ground.n[2] = -1; ground.d = r.uni(1.2, 2.0);
  s.planes.push_back(ground);
  int ne = 4 + (int)(r.next() % 13);
  for (int i = 0; i < ne; ++i) {
    double a = r.uni(0, 2 * M_PI), d = r.uni(3, 20);
    double cx = d * std::cos(a), cy = d * std::sin(a), w = r.uni(0.1, 0.3);
    if (r.next() & 1) {
      add_box(s, cx - w, cy - w, -3, cx + w, cy + w, 8);              // vertical edge
    } else {
      double l = r.uni(2, 8), zc = r.uni(-1, 4);
      if (r.next() & 1) add_box(s, cx - l, cy - w, zc - w, cx + l, cy + w, zc + w);
      else add_box(s, cx - w, cy - l, zc - w, cx + w, cy + l, zc + w);
    }
  }
}

inline bool ray_box(const double o[3], const double d[3], const Box& b, double& t) {
  double tn = -1e300, tf = 1e300;
  for (int k = 0; k < 3; ++k) {
    if (std::fabs(d[k]) < 1e-15) {
      if (o[k] < b.lo[k] || o[k] > b.hi[k]) return false;
      continue;
    }
    double inv = 1.0 / d[k];
    double t0 = (b.lo[k] - o[k]) * inv, t1 = (b.hi[k] - o[k]) * inv;
    if (t0 > t1) { double q = t0; t0 = t1; t1 = q; }
    if (t0 > tn) tn = t0;
    if (t1 < tf) tf = t1;
    if (tn > tf) return false;
  }
  if (tn > 1e-6) { t = tn; return true; }
  if (tf > 1e-6) { t = tf; return true; }
  return false;
}

inline bool ray_plane(const double o[3], const double d[3], const Plane& p, double& t) {
  double den = p.n[0] * d[0] + p.n[1] * d[1] + p.n[2] * d[2];
  if (std::fabs(den) < 1e-12) return false;
  double tt = (p.d - (p.n[0] * o[0] + p.n[1] * o[1] + p.n[2] * o[2])) / den;
  if (tt <= 1e-6) return false;
  t = tt;
  return true;
}

double cast(const Scene& s, const double o[3], const double d[3]) {
  double best = 1e300, t;
  for (const Box& b : s.boxes)
    if (ray_box(o, d, b, t) && t < best) best = t;
  for (const Plane& p : s.planes)
    if (ray_plane(o, d, p, t) && t < best) best = t;
  return best;
}

struct Lidar {
  int n_lasers, cols;
  double elev[64];
  double period, fire_dt;
};

Lidar make_lidar(int kind) {
  Lidar L;
  std::memset(&L, 0, sizeof(L));
  L.period = 0.1;
  if (kind == SYNTH_HDL64) {
    L.n_lasers = 64;
    L.cols = 2048;
    for (int k = 0; k < 64; ++k) L.elev[k] = -24.8 + (2.0 + 24.8) * k / 63.0;
    L.fire_dt = 0.1 / 2048 / 64;
  } else {
    // VLP-16 firing order: -15, 1, -13, 3, ..., -1, 15 degrees
    L.n_lasers = 16;
    L.cols = 1800;
    for (int k = 0; k < 16; ++k) L.elev[k] = (k % 2 == 0) ? (-15.0 + k) : (k - 0.0);
    L.fire_dt = 2.304e-6;
  }
  return L;
}

// pose = (x, y, z, roll, pitch, yaw); R = Rz(yaw) Ry(pitch) Rx(roll)
void pose_apply(const double pose[6], const double v[3], double out[3]) {
  double cr = std::cos(pose[3]), sr = std::sin(pose[3]);
  double cp = std::cos(pose[4]), sp = std::sin(pose[4]);
  double cy = std::cos(pose[5]), sy = std::sin(pose[5]);
  double x1 = v[0], y1 = cr * v[1] - sr * v[2], z1 = sr * v[1] + cr * v[2];
  double x2 = cp * x1 + sp * z1, y2 = y1, z2 = -sp * x1 + cp * z1;
  out[0] = cy * x2 - sy * y2;
  out[1] = sy * x2 + cy * y2;
  out[2] = z2;
}

int sweep(const Scene& sc, int lidar, const double* p0, const double* p1, uint64_t seed,
          double sigma, double start_az, float* out, int cap) {
  Lidar L = make_lidar(lidar);
  Rng rng(seed);
  int n = 0;
  const double max_range = 100.0, min_range = 0.3;
  for (int c = 0; c < L.cols; ++c) {
    for (int k = 0; k < L.n_lasers; ++k) {
      double tau = (double)c * (L.period / L.cols) + (double)k * L.fire_dt;
      double f = tau / L.period;
      double pose[6];
      for (int q = 0; q < 6; ++q) pose[q] = p0[q] + (p1[q] - p0[q]) * f;
      double az = start_az - 2.0 * M_PI * f;
      double el = L.elev[k] * M_PI / 180.0;
      double dl[3] = {std::cos(el) * std::cos(az), std::cos(el) * std::sin(az), std::sin(el)};
      double dw[3];
      pose_apply(pose, dl, dw);
      double t = cast(sc, pose, dw);
      double noise = rng.gauss() * sigma;
      if (t > max_range || t < min_range) continue;
      double r = t + noise;
      if (n >= cap) return -1;
      out[4 * n + 0] = (float)(r * dl[0]);
      out[4 * n + 1] = (float)(r * dl[1]);
      out[4 * n + 2] = (float)(r * dl[2]);
      out[4 * n + 3] = (float)k;
      ++n;
    }
  }
  return n;
}

}  // namespace

extern "C" {

void* synth_scene_create(int kind, uint64_t seed) {
  Scene* s = new Scene();
  if (kind == SYNTH_SCENE_RANDOM) build_random(*s, seed);
  else build_indoor(*s, seed);
  return s;
}

void synth_scene_destroy(void* s) { delete static_cast<Scene*>(s); }

int synth_max_points(int lidar) {
  Lidar L = make_lidar(lidar);
  return L.n_lasers * L.cols;
}

int synth_sweep(const void* scene, int lidar, const double pose0[6], const double pose1[6],
                uint64_t noise_seed, double sigma, double start_az, float* out, int cap) {
  return sweep(*static_cast<const Scene*>(scene), lidar, pose0, pose1, noise_seed, sigma,
               start_az, out, cap);
}

int synth_batch(int n, const void* const* scenes, int lidar, const double* poses0,
                const double* poses1, const uint64_t* seeds, double sigma, double start_az,
                float* out, int cap_per_sweep, int* counts, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  std::vector<int> bad(nthreads, 0);
  for (int w = 0; w < nthreads; ++w) {
    th.emplace_back([=, &bad]() {
      for (int i = w; i < n; i += nthreads) {
        int c = sweep(*static_cast<const Scene*>(scenes[i]), lidar, poses0 + 6 * i,
                      poses1 + 6 * i, seeds[i], sigma, start_az,
                      out + (size_t)4 * cap_per_sweep * i, cap_per_sweep);
        counts[i] = c;
        if (c < 0) bad[w] = 1;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int w = 0; w < nthreads; ++w)
    if (bad[w]) return -1;
  return 0;
}

}  // extern "C"
