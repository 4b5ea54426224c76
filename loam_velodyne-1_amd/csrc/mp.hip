// Laser mapping on gfx950 (placeholder until the mapping kernels land).
#include "mp.hpp"

namespace loam {

void mp_alloc(MpBuffers& b, int P, int, int, int, int) { b.P = P; }
void mp_free(MpBuffers& b) { b = MpBuffers(); }
int mp_stream_frame(MpBuffers&, hipStream_t, const loam_pose6&, const loam_cloud_out&, const loam_cloud_out&,
                    const loam_cloud_out&, loam_pose6*, loam_pose6*, loam_cloud_out*, loam_stats*, std::string& err) {
  err = "mapping kernels not built yet";
  return LOAM_E_INVAL;
}
void mp_batch_run(MpBuffers&, const OdBuffers&, hipStream_t) {}
int mp_batch_download(MpBuffers& b, hipStream_t, loam_pose6* aft, loam_stats*, std::string&) {
  if (aft)
    for (int i = 0; i < b.P; ++i) aft[i] = loam_pose6{0, 0, 0, 0, 0, 0};
  return LOAM_OK;
}

}  // namespace loam
