// Mapping device buffers and entry points (engine-internal).
#ifndef LOAM_MP_HPP
#define LOAM_MP_HPP

#include <hip/hip_runtime.h>

#include <string>

#include "engine.hpp"
#include "od.hpp"

namespace loam {

struct MpBuffers {
  int P = 0;
};

inline int mp_batch_map_capacity(int cap) { return 4 * cap; }
void mp_alloc(MpBuffers& b, int P, int R, int cap_pts, int map_cap, int max_iter);
void mp_free(MpBuffers& b);
int mp_stream_frame(MpBuffers& b, hipStream_t st, const loam_pose6& odom_sum, const loam_cloud_out& corner,
                    const loam_cloud_out& surf, const loam_cloud_out& full, loam_pose6* aft, loam_pose6* bef,
                    loam_cloud_out* registered, loam_stats* stats, std::string& err);
void mp_batch_run(MpBuffers& b, const OdBuffers& od, hipStream_t st);
int mp_batch_download(MpBuffers& b, hipStream_t st, loam_pose6* aft, loam_stats* stats, std::string& err);

}  // namespace loam
#endif
