// Streaming node path driven from C++ through the C-ABI (include/loam/loam.h), the way a ROS node
// wrapper would call it: preallocated caller-owned buffers, one sweep at a time,
// loam_scan_registration -> loam_odometry -> loam_mapping on the frames odometry publishes.
// Reads sweeps written by tools/stream_node.py (u32 count, then count x 4 floats, per sweep) and
// prints one JSON line with the per-stage wall times.  Measures the engine without the Python
// binding's per-call allocations.
//
//   g++ -O2 -std=c++17 tools/stream_node.cpp -I include -L loam_velodyne-1_amd -lloam_hip \
//       -Wl,-rpath,$PWD/loam_velodyne-1_amd -o tools/stream_node
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "loam/loam.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: stream_node SWEEPS.bin [system_delay]\n");
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<std::vector<loam_point>> sweeps;
  uint32_t n;
  while (std::fread(&n, 4, 1, f) == 1) {
    sweeps.emplace_back(n);
    if (std::fread(sweeps.back().data(), sizeof(loam_point), n, f) != n) return 2;
  }
  std::fclose(f);
  loam_config cfg;
  loam_config_default(&cfg);
  if (argc > 2) cfg.system_delay = (uint32_t)std::atoi(argv[2]);
  loam_ctx* ctx = nullptr;
  if (loam_create(&ctx, &cfg, 0) != LOAM_OK) {
    std::fprintf(stderr, "loam_create: %s\n", loam_last_error());
    return 1;
  }
  const uint32_t cap = cfg.max_points;
  std::vector<loam_point> full(cap), sharp(cap), lsharp(cap), flat(cap), lflat(cap), cl(cap), sl(cap), fe(cap), reg(cap);
  loam_features feat;
  auto out = [](std::vector<loam_point>& v) { return loam_cloud_out{v.data(), 0, (uint32_t)v.size()}; };
  double t_sr = 0, t_od = 0, t_mp = 0;
  int processed = 0, mapped = 0;
  loam_pose6 last_aft{};
  for (size_t k = 0; k < sweeps.size(); ++k) {
    feat.full = out(full); feat.sharp = out(sharp); feat.less_sharp = out(lsharp);
    feat.flat = out(flat); feat.less_flat = out(lflat);
    const double stamp = 0.1 * (double)k;
    loam_cloud_in in{sweeps[k].data(), (uint32_t)sweeps[k].size(), sizeof(loam_point)};
    const double a = now();
    int rc = loam_scan_registration(ctx, stamp, in, &feat);
    const double b = now();
    t_sr += b - a;
    if (rc == LOAM_E_NOT_READY) continue;
    if (rc != LOAM_OK) { std::fprintf(stderr, "sr: %s\n", loam_last_error()); return 1; }
    ++processed;
    loam_pose6 sum;
    loam_cloud_out c1 = out(cl), c2 = out(sl), c3 = out(fe);
    int pub = 0;
    rc = loam_odometry(ctx, stamp, &feat, &sum, &c1, &c2, &c3, &pub);
    const double c = now();
    t_od += c - b;
    if (rc != LOAM_OK) { std::fprintf(stderr, "od: %s\n", loam_last_error()); return 1; }
    if (pub == (LOAM_PUB_POSE | LOAM_PUB_CLOUDS | LOAM_PUB_FULL)) {
      loam_pose6 aft, bef;
      loam_cloud_out r = out(reg);
      rc = loam_mapping(ctx, stamp, &sum, &c1, &c2, &c3, &aft, &bef, &r);
      if (rc != LOAM_OK) { std::fprintf(stderr, "mp: %s\n", loam_last_error()); return 1; }
      last_aft = aft;
      ++mapped;
    }
    t_mp += now() - c;
  }
  loam_destroy(ctx);
  const double tot = t_sr + t_od + t_mp;
  std::printf("{\"sweeps_processed\": %d, \"mapping_frames\": %d, \"scans_per_s\": %.3f, \"ms_per_sweep\": %.4f, "
              "\"ms_sr\": %.4f, \"ms_od\": %.4f, \"ms_mp_per_processed\": %.4f, \"final_aft\": [%.6g, %.6g, %.6g, %.6g, %.6g, %.6g]}\n",
              processed, mapped, processed / tot, 1e3 * tot / processed, 1e3 * t_sr / processed, 1e3 * t_od / processed,
              1e3 * t_mp / processed, last_aft.rx, last_aft.ry, last_aft.rz, last_aft.tx, last_aft.ty, last_aft.tz);
  return 0;
}
