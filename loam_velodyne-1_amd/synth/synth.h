// Synthetic lidar sweep generator: C ABI (test and bench input only; see synth.cpp).
#ifndef LOAM_SYNTH_H
#define LOAM_SYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { SYNTH_SCENE_INDOOR = 0, SYNTH_SCENE_RANDOM = 1 };
enum { SYNTH_VLP16 = 0, SYNTH_HDL64 = 1 };

void* synth_scene_create(int kind, uint64_t seed);
void synth_scene_destroy(void* scene);
int synth_max_points(int lidar);
/* pose = (x, y, z, roll, pitch, yaw) in the world frame (x fwd, y left, z up) at sweep start
   (pose0) and sweep end (pose1); output = float4 (x, y, z, laser) in the instantaneous sensor
   frame, firing order.  Returns the point count, or -1 if cap is too small. */
int synth_sweep(const void* scene, int lidar, const double pose0[6], const double pose1[6],
                uint64_t noise_seed, double sigma, double start_az, float* out, int cap);
int synth_batch(int n, const void* const* scenes, int lidar, const double* poses0,
                const double* poses1, const uint64_t* seeds, double sigma, double start_az,
                float* out, int cap_per_sweep, int* counts, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
