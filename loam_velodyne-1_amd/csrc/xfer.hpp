// Small host <-> device transfers of a node call in one launch (engine-internal).  A node call moves
// a handful of scalars each way (counts, poses, the L-M state): as separate hipMemcpyAsync calls each
// was a ~4 us copy on the stream (config 3 chain: 13 per sweep).  k_xfer writes host values carried
// in its arguments to device memory (put) and copies device words into the context's mapped,
// coherent host block (get), all in one one-workgroup launch.
#ifndef LOAM_XFER_HPP
#define LOAM_XFER_HPP

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>

namespace loam {

struct Xfer {
  static constexpr int kMax = 8, kImm = 64;
  int n = 0, nimm = 0;
  bool overflow = false;  // an entry did not fit: xfer_launch refuses the whole transfer
  uint32_t* dst[kMax];
  const uint32_t* src[kMax];  // nullptr: a put from imm
  int words[kMax], imm_off[kMax];
  uint32_t imm[kImm];
  // device words <- host bytes (a multiple of 4), copied into the launch's arguments now
  bool put(void* dev, const void* host, int nbytes) {
    const int w = nbytes / 4;
    if (n == kMax || nimm + w > kImm || nbytes % 4) {
      overflow = true;
      return false;
    }
    dst[n] = (uint32_t*)dev;
    src[n] = nullptr;
    words[n] = w;
    imm_off[n] = nimm;
    std::memcpy(imm + nimm, host, (size_t)w * 4);
    nimm += w;
    ++n;
    return true;
  }
  // mapped host words (the device address of the context's host block) <- device bytes
  bool get(void* host_dev, const void* dev, int nbytes) {
    if (n == kMax || nbytes % 4) {
      overflow = true;
      return false;
    }
    dst[n] = (uint32_t*)host_dev;
    src[n] = (const uint32_t*)dev;
    words[n] = nbytes / 4;
    imm_off[n] = 0;
    ++n;
    return true;
  }
};

// the context's mapped host block: h for the host, d for kernels (the same memory)
struct XferBuf {
  char* h = nullptr;
  char* d = nullptr;
};

// hipErrorInvalidValue (nothing launched) when an entry did not fit, else the launch's error
hipError_t xfer_launch(const Xfer& x, hipStream_t st);

// what a streaming node call needs beyond its buffers: the pinned scratch (meta), the mapped host
// block (xb; regions: scan registration [0, 64), odometry [64, 512), mapping [512, 1024) bytes) and
// two timing events of the context
struct StreamIo {
  void* meta = nullptr;
  XferBuf xb;
  hipEvent_t e0 = nullptr, e1 = nullptr;
};
constexpr int kXferSr = 0, kXferOd = 64, kXferMp = 512, kXferMpUpd = 1024, kXferBytes = 4096;

}  // namespace loam

#endif
