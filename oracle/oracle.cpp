// ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference hot path, used by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline as the checker and the timed CPU baseline.
// The product (libloam_hip.so) never links, loads or calls anything in oracle/.
//
// PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors and it
// cannot be built here (PCL 1.7 / OpenCV 2.4 / ROS are absent; building it against stand-in
// headers is not allowed), so this restatement is checked against hand-derived known answers and
// independent numpy computations only (tests/test_oracle_*.py).
//
// Follows, line by line (every quirk of SURVEY.md appendix A1):
//   scan registration   /root/reference/src/scanRegistration.cpp:211-636
//   odometry            /root/reference/src/laserOdometry.cpp:101-273, 413-931
//   mapping             /root/reference/src/laserMapping.cpp:110-272, 408-1097
//   maintenance         /root/reference/src/transformMaintenance.cpp:60-203
//
// Numerics model = the reference's own toolchain (ROS Indigo: GCC 4.8 + glibc, x86-64 SSE, no FMA;
// build with -ffp-contract=off):
//   * scanRegistration.cpp has `using std::sin/cos/atan2` (:51-53): float overloads for those;
//   * every other unqualified libm call (sqrt, atan, asin, fabs, pow, and sin/cos/atan2 in the
//     other three files) binds the C double function, so the expression around it is evaluated in
//     double and rounded once on assignment to float — written here with explicit (double) casts;
//   * double literals (0.1, 1.8, 25.0, M_PI, ...) promote their expression to double.
// IMU input (§8f rank 1) is modelled: scanRegistration's imuHandler queue, per-point de-skew and
// /imu_trans (src/scanRegistration.cpp:68-209, 286-349, 614-660), the odometry IMU terms
// (src/laserOdometry.cpp:196-254, 330-354) and the mapping roll / pitch blend
// (src/laserMapping.cpp:199-226, 323-335).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

#include "../include/loam/loam.h"
#include "oracle_math.hpp"

using namespace oracle;

namespace {

inline double D(float x) { return (double)x; }
inline double dsin(float x) { return std::sin((double)x); }
inline double dcos(float x) { return std::cos((double)x); }
inline double rad2deg(double r) { return r * 180.0 / M_PI; }  // include/loam_velodyne/common.h:39

struct Cfg {
  int n_rings, ring_model;
  float ring_lo, ring_hi;
  int system_delay, od_max_iter, mp_max_iter, skip_frame_num;
};

Cfg make_cfg(const loam_config* c) {
  loam_config d;
  if (c == nullptr) {
    std::memset(&d, 0, sizeof(d));
    d.n_rings = 16; d.ring_model = LOAM_RING_VLP16; d.ring_lo_deg = -24.8f; d.ring_hi_deg = 2.0f;
    d.system_delay = 20; d.max_points = 40000; d.od_max_iter = 25; d.mp_max_iter = 10;
    d.skip_frame_num = 1;
    c = &d;
  }
  Cfg g;
  g.n_rings = (int)c->n_rings; g.ring_model = (int)c->ring_model;
  g.ring_lo = c->ring_lo_deg; g.ring_hi = c->ring_hi_deg;
  g.system_delay = (int)c->system_delay; g.od_max_iter = (int)c->od_max_iter;
  g.mp_max_iter = (int)c->mp_max_iter; g.skip_frame_num = (int)c->skip_frame_num;
  return g;
}

// ===================================================================== scan registration
struct SrOut {
  std::vector<P> full, sharp, lsharp, flat, lflat;
  float imu_trans[12] = {0};  // /imu_trans (:614-635)
};

// src/scanRegistration.cpp:248-260 (VLP-16) and the bk HDL-64E hint (bk :268-275)
int ring_id(const Cfg& c, float angle) {
  if (c.ring_model == LOAM_RING_LINEAR) {
    const float step = (c.ring_hi - c.ring_lo) / (float)(c.n_rings - 1);
    const float angleID = (angle - c.ring_lo) / step;
    return (int)(angleID + 0.5f);
  }
  int rounded = (int)(D(angle) + (D(angle) < 0.0 ? -0.5 : +0.5));
  return rounded > 0 ? rounded : rounded + (c.n_rings - 1);
}

// laserCloudHandler body after the systemDelay gate: src/scanRegistration.cpp:221-581
// scanRegistration's IMU globals (src/scanRegistration.cpp:68-97), fed by imuHandler (:638-660)
constexpr int kImuQue = 200;  // imuQueLength
struct SrImu {
  int front = 0, last = -1;
  float rollStart = 0, pitchStart = 0, yawStart = 0, rollCur = 0, pitchCur = 0, yawCur = 0;
  float veloXStart = 0, veloYStart = 0, veloZStart = 0, shiftXStart = 0, shiftYStart = 0, shiftZStart = 0;
  float veloXCur = 0, veloYCur = 0, veloZCur = 0, shiftXCur = 0, shiftYCur = 0, shiftZCur = 0;
  float shiftFSX = 0, shiftFSY = 0, shiftFSZ = 0, veloFSX = 0, veloFSY = 0, veloFSZ = 0;
  double time[kImuQue] = {0};
  float roll[kImuQue] = {0}, pitch[kImuQue] = {0}, yaw[kImuQue] = {0};
  float accX[kImuQue] = {0}, accY[kImuQue] = {0}, accZ[kImuQue] = {0};
  float veloX[kImuQue] = {0}, veloY[kImuQue] = {0}, veloZ[kImuQue] = {0};
  float shiftX[kImuQue] = {0}, shiftY[kImuQue] = {0}, shiftZ[kImuQue] = {0};
};

// float std::sin / std::cos: scanRegistration's `using std::sin; using std::cos;` (:51-52) binds the
// float overloads for float arguments
inline float fsin(float x) { return std::sin(x); }
inline float fcos(float x) { return std::cos(x); }

// :162-200 AccumulateIMUShift
void accumulate_imu_shift(SrImu& m) {
  const int L = m.last;
  float roll = m.roll[L], pitch = m.pitch[L], yaw = m.yaw[L];
  float accX = m.accX[L], accY = m.accY[L], accZ = m.accZ[L];
  float x1 = fcos(roll) * accX - fsin(roll) * accY;
  float y1 = fsin(roll) * accX + fcos(roll) * accY;
  float z1 = accZ;
  float x2 = x1;
  float y2 = fcos(pitch) * y1 - fsin(pitch) * z1;
  float z2 = fsin(pitch) * y1 + fcos(pitch) * z1;
  accX = fcos(yaw) * x2 + fsin(yaw) * z2;
  accY = y2;
  accZ = -fsin(yaw) * x2 + fcos(yaw) * z2;
  const int B = (L + kImuQue - 1) % kImuQue;
  double timeDiff = m.time[L] - m.time[B];
  if (timeDiff < 0.1) {  // scanPeriod (double, :55)
    m.shiftX[L] = (float)(D(m.shiftX[B]) + D(m.veloX[B]) * timeDiff + D(accX) * timeDiff * timeDiff / 2);
    m.shiftY[L] = (float)(D(m.shiftY[B]) + D(m.veloY[B]) * timeDiff + D(accY) * timeDiff * timeDiff / 2);
    m.shiftZ[L] = (float)(D(m.shiftZ[B]) + D(m.veloZ[B]) * timeDiff + D(accZ) * timeDiff * timeDiff / 2);
    m.veloX[L] = (float)(D(m.veloX[B]) + D(accX) * timeDiff);
    m.veloY[L] = (float)(D(m.veloY[B]) + D(accY) * timeDiff);
    m.veloZ[L] = (float)(D(m.veloZ[B]) + D(accZ) * timeDiff);
  }
}

// :638-660 imuHandler
void sr_imu_handler(SrImu& m, double stamp, const double* q, const double* acc) {
  double roll, pitch, yaw;
  tf_get_rpy(Quat{q[0], q[1], q[2], q[3]}, roll, pitch, yaw);
  float accX = (float)(acc[1] - std::sin(roll) * std::cos(pitch) * 9.81);
  float accY = (float)(acc[2] - std::cos(roll) * std::cos(pitch) * 9.81);
  float accZ = (float)(acc[0] + std::sin(pitch) * 9.81);
  m.last = (m.last + 1) % kImuQue;
  m.time[m.last] = stamp;
  m.roll[m.last] = (float)roll;
  m.pitch[m.last] = (float)pitch;
  m.yaw[m.last] = (float)yaw;
  m.accX[m.last] = accX;
  m.accY[m.last] = accY;
  m.accZ[m.last] = accZ;
  accumulate_imu_shift(m);
}

// :111-127 ShiftToStartIMU
void shift_to_start_imu(SrImu& m, float pointTime) {
  m.shiftFSX = m.shiftXCur - m.shiftXStart - m.veloXStart * pointTime;
  m.shiftFSY = m.shiftYCur - m.shiftYStart - m.veloYStart * pointTime;
  m.shiftFSZ = m.shiftZCur - m.shiftZStart - m.veloZStart * pointTime;
  float x1 = fcos(m.yawStart) * m.shiftFSX - fsin(m.yawStart) * m.shiftFSZ;
  float y1 = m.shiftFSY;
  float z1 = fsin(m.yawStart) * m.shiftFSX + fcos(m.yawStart) * m.shiftFSZ;
  float x2 = x1;
  float y2 = fcos(m.pitchStart) * y1 + fsin(m.pitchStart) * z1;
  float z2 = -fsin(m.pitchStart) * y1 + fcos(m.pitchStart) * z1;
  m.shiftFSX = fcos(m.rollStart) * x2 + fsin(m.rollStart) * y2;
  m.shiftFSY = -fsin(m.rollStart) * x2 + fcos(m.rollStart) * y2;
  m.shiftFSZ = z2;
}

// :129-145 VeloToStartIMU
void velo_to_start_imu(SrImu& m) {
  m.veloFSX = m.veloXCur - m.veloXStart;
  m.veloFSY = m.veloYCur - m.veloYStart;
  m.veloFSZ = m.veloZCur - m.veloZStart;
  float x1 = fcos(m.yawStart) * m.veloFSX - fsin(m.yawStart) * m.veloFSZ;
  float y1 = m.veloFSY;
  float z1 = fsin(m.yawStart) * m.veloFSX + fcos(m.yawStart) * m.veloFSZ;
  float x2 = x1;
  float y2 = fcos(m.pitchStart) * y1 + fsin(m.pitchStart) * z1;
  float z2 = -fsin(m.pitchStart) * y1 + fcos(m.pitchStart) * z1;
  m.veloFSX = fcos(m.rollStart) * x2 + fsin(m.rollStart) * y2;
  m.veloFSY = -fsin(m.rollStart) * x2 + fcos(m.rollStart) * y2;
  m.veloFSZ = z2;
}

// :147-160 TransformToStartIMU
void transform_to_start_imu(const SrImu& m, P& p) {
  float x1 = fcos(m.rollCur) * p.x - fsin(m.rollCur) * p.y;
  float y1 = fsin(m.rollCur) * p.x + fcos(m.rollCur) * p.y;
  float z1 = p.z;
  float x2 = x1;
  float y2 = fcos(m.pitchCur) * y1 - fsin(m.pitchCur) * z1;
  float z2 = fsin(m.pitchCur) * y1 + fcos(m.pitchCur) * z1;
  float x3 = fcos(m.yawCur) * x2 + fsin(m.yawCur) * z2;
  float y3 = y2;
  float z3 = -fsin(m.yawCur) * x2 + fcos(m.yawCur) * z2;
  float x4 = fcos(m.yawStart) * x3 - fsin(m.yawStart) * z3;
  float y4 = y3;
  float z4 = fsin(m.yawStart) * x3 + fcos(m.yawStart) * z3;
  float x5 = x4;
  float y5 = fcos(m.pitchStart) * y4 + fsin(m.pitchStart) * z4;
  float z5 = -fsin(m.pitchStart) * y4 + fcos(m.pitchStart) * z4;
  p.x = fcos(m.rollStart) * x5 + fsin(m.rollStart) * y5 + m.shiftFSX;
  p.y = -fsin(m.rollStart) * x5 + fcos(m.rollStart) * y5 + m.shiftFSY;
  p.z = z5 + m.shiftFSZ;
}

// :286-349 the per-point IMU block
void sr_point_imu(SrImu& m, double timeScanCur, float relTime, int i, P& point) {
  float pointTime = (float)(D(relTime) * 0.1);  // scanPeriod (double)
  while (m.front != m.last) {
    if (timeScanCur + pointTime < m.time[m.front]) break;
    m.front = (m.front + 1) % kImuQue;
  }
  const int F = m.front;
  if (timeScanCur + pointTime > m.time[F]) {
    m.rollCur = m.roll[F]; m.pitchCur = m.pitch[F]; m.yawCur = m.yaw[F];
    m.veloXCur = m.veloX[F]; m.veloYCur = m.veloY[F]; m.veloZCur = m.veloZ[F];
    m.shiftXCur = m.shiftX[F]; m.shiftYCur = m.shiftY[F]; m.shiftZCur = m.shiftZ[F];
  } else {
    const int B = (F + kImuQue - 1) % kImuQue;
    float ratioFront = (float)((timeScanCur + pointTime - m.time[B]) / (m.time[F] - m.time[B]));
    float ratioBack = (float)((m.time[F] - timeScanCur - pointTime) / (m.time[F] - m.time[B]));
    m.rollCur = m.roll[F] * ratioFront + m.roll[B] * ratioBack;
    m.pitchCur = m.pitch[F] * ratioFront + m.pitch[B] * ratioBack;
    if (D(m.yaw[F] - m.yaw[B]) > M_PI)
      m.yawCur = (float)(D(m.yaw[F] * ratioFront) + (D(m.yaw[B]) + 2 * M_PI) * D(ratioBack));
    else if (D(m.yaw[F] - m.yaw[B]) < -M_PI)
      m.yawCur = (float)(D(m.yaw[F] * ratioFront) + (D(m.yaw[B]) - 2 * M_PI) * D(ratioBack));
    else
      m.yawCur = m.yaw[F] * ratioFront + m.yaw[B] * ratioBack;
    m.veloXCur = m.veloX[F] * ratioFront + m.veloX[B] * ratioBack;
    m.veloYCur = m.veloY[F] * ratioFront + m.veloY[B] * ratioBack;
    m.veloZCur = m.veloZ[F] * ratioFront + m.veloZ[B] * ratioBack;
    m.shiftXCur = m.shiftX[F] * ratioFront + m.shiftX[B] * ratioBack;
    m.shiftYCur = m.shiftY[F] * ratioFront + m.shiftY[B] * ratioBack;
    m.shiftZCur = m.shiftZ[F] * ratioFront + m.shiftZ[B] * ratioBack;
  }
  if (i == 0) {
    m.rollStart = m.rollCur; m.pitchStart = m.pitchCur; m.yawStart = m.yawCur;
    m.veloXStart = m.veloXCur; m.veloYStart = m.veloYCur; m.veloZStart = m.veloZCur;
    m.shiftXStart = m.shiftXCur; m.shiftYStart = m.shiftYCur; m.shiftZStart = m.shiftZCur;
  } else {
    shift_to_start_imu(m, pointTime);
    velo_to_start_imu(m);
    transform_to_start_imu(m, point);
  }
}

int sr_body(const Cfg& cfg, const float* raw, size_t n, size_t stride_f, SrOut& o, SrImu& imu,
            double timeScanCur) {
  const int N = cfg.n_rings;
  // fromROSMsg + removeNaNFromPointCloud (:225-228)
  std::vector<P> in;
  in.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    const float* r = raw + i * stride_f;
    if (std::isfinite(r[0]) && std::isfinite(r[1]) && std::isfinite(r[2]))
      in.push_back(P{r[0], r[1], r[2], 0.0f});
  }
  int cloudSize = (int)in.size();
  if (cloudSize == 0) return LOAM_E_INVAL;
  // :230-238
  float startOri = -std::atan2(in[0].y, in[0].x);
  float endOri = (float)(D(-std::atan2(in[cloudSize - 1].y, in[cloudSize - 1].x)) + 2 * M_PI);
  if (D(endOri - startOri) > 3 * M_PI) endOri = (float)(D(endOri) - 2 * M_PI);
  else if (D(endOri - startOri) < M_PI) endOri = (float)(D(endOri) + 2 * M_PI);

  // :239-351 ring / time loop
  bool halfPassed = false;
  int count = cloudSize;
  std::vector<std::vector<P>> scans(N);
  for (int i = 0; i < cloudSize; ++i) {
    P point;
    point.x = in[i].y;
    point.y = in[i].z;
    point.z = in[i].x;
    float angle = (float)(std::atan(D(point.y) / std::sqrt(D(point.x * point.x + point.z * point.z))) *
                          180 / M_PI);
    int scanID = ring_id(cfg, angle);
    if (scanID > (N - 1) || scanID < 0) { count--; continue; }
    float ori = -std::atan2(point.x, point.z);
    if (!halfPassed) {
      if (D(ori) < D(startOri) - M_PI / 2) ori = (float)(D(ori) + 2 * M_PI);
      else if (D(ori) > D(startOri) + M_PI * 3 / 2) ori = (float)(D(ori) - 2 * M_PI);
      if (D(ori - startOri) > M_PI) halfPassed = true;
    } else {
      ori = (float)(D(ori) + 2 * M_PI);
      if (D(ori) < D(endOri) - M_PI * 3 / 2) ori = (float)(D(ori) + 2 * M_PI);
      else if (D(ori) > D(endOri) + M_PI / 2) ori = (float)(D(ori) - 2 * M_PI);
    }
    float relTime = (ori - startOri) / (endOri - startOri);
    point.intensity = (float)(scanID + 0.1 * D(relTime));   // scanPeriod is double here (:55)
    if (imu.last >= 0) sr_point_imu(imu, timeScanCur, relTime, i, point);  // :286-349
    scans[scanID].push_back(point);
  }
  cloudSize = count;

  // :614-635 /imu_trans: start RPY (as pitch, yaw, roll), current RPY, shift and velocity from start
  const float it[12] = {imu.pitchStart, imu.yawStart, imu.rollStart, imu.pitchCur, imu.yawCur, imu.rollCur,
                        imu.shiftFSX, imu.shiftFSY, imu.shiftFSZ, imu.veloFSX, imu.veloFSY, imu.veloFSZ};
  std::memcpy(o.imu_trans, it, sizeof(it));

  // :354-357 concat rings
  std::vector<P>& lc = o.full;
  lc.clear();
  for (int r = 0; r < N; ++r) lc.insert(lc.end(), scans[r].begin(), scans[r].end());

  // per-call state (the reference keeps these in static arrays; reset over the whole cloud here)
  std::vector<float> curv(cloudSize, 0.0f);
  std::vector<int> sortInd(cloudSize), picked(cloudSize, 0), label(cloudSize, 0);
  std::iota(sortInd.begin(), sortInd.end(), 0);
  std::vector<int> startInd(N, 0), endInd(N, 0);

  // :358-393 curvature + ring bounds
  int scanCount = -1;
  for (int i = 5; i < cloudSize - 5; ++i) {
    float dX = lc[i - 5].x + lc[i - 4].x + lc[i - 3].x + lc[i - 2].x + lc[i - 1].x - 10 * lc[i].x +
               lc[i + 1].x + lc[i + 2].x + lc[i + 3].x + lc[i + 4].x + lc[i + 5].x;
    float dY = lc[i - 5].y + lc[i - 4].y + lc[i - 3].y + lc[i - 2].y + lc[i - 1].y - 10 * lc[i].y +
               lc[i + 1].y + lc[i + 2].y + lc[i + 3].y + lc[i + 4].y + lc[i + 5].y;
    float dZ = lc[i - 5].z + lc[i - 4].z + lc[i - 3].z + lc[i - 2].z + lc[i - 1].z - 10 * lc[i].z +
               lc[i + 1].z + lc[i + 2].z + lc[i + 3].z + lc[i + 4].z + lc[i + 5].z;
    curv[i] = dX * dX + dY * dY + dZ * dZ;
    sortInd[i] = i;
    picked[i] = 0;
    label[i] = 0;
    if ((int)lc[i].intensity != scanCount) {
      scanCount = (int)lc[i].intensity;
      if (scanCount > 0 && scanCount < N) {
        startInd[scanCount] = i + 5;
        endInd[scanCount - 1] = i - 5;
      }
    }
  }
  startInd[0] = 5;
  endInd[N - 1] = cloudSize - 5;

  // :395-452 occlusion / parallel-beam marking
  for (int i = 5; i < cloudSize - 6; ++i) {
    float dX = lc[i + 1].x - lc[i].x, dY = lc[i + 1].y - lc[i].y, dZ = lc[i + 1].z - lc[i].z;
    float diff = dX * dX + dY * dY + dZ * dZ;
    if (D(diff) > 0.1) {
      float depth1 = (float)std::sqrt(D(lc[i].x * lc[i].x + lc[i].y * lc[i].y + lc[i].z * lc[i].z));
      float depth2 = (float)std::sqrt(
          D(lc[i + 1].x * lc[i + 1].x + lc[i + 1].y * lc[i + 1].y + lc[i + 1].z * lc[i + 1].z));
      if (depth1 > depth2) {
        dX = lc[i + 1].x - lc[i].x * depth2 / depth1;
        dY = lc[i + 1].y - lc[i].y * depth2 / depth1;
        dZ = lc[i + 1].z - lc[i].z * depth2 / depth1;
        if (std::sqrt(D(dX * dX + dY * dY + dZ * dZ)) / D(depth2) < 0.1)
          for (int k = i - 5; k <= i; ++k) picked[k] = 1;
      } else {
        dX = lc[i + 1].x * depth1 / depth2 - lc[i].x;
        dY = lc[i + 1].y * depth1 / depth2 - lc[i].y;
        dZ = lc[i + 1].z * depth1 / depth2 - lc[i].z;
        if (std::sqrt(D(dX * dX + dY * dY + dZ * dZ)) / D(depth1) < 0.1)
          for (int k = i + 1; k <= i + 6; ++k) picked[k] = 1;
      }
    }
    float dX2 = lc[i].x - lc[i - 1].x, dY2 = lc[i].y - lc[i - 1].y, dZ2 = lc[i].z - lc[i - 1].z;
    float diff2 = dX2 * dX2 + dY2 * dY2 + dZ2 * dZ2;
    float dis = lc[i].x * lc[i].x + lc[i].y * lc[i].y + lc[i].z * lc[i].z;
    if (D(diff) > 0.0002 * D(dis) && D(diff2) > 0.0002 * D(dis)) picked[i] = 1;
  }

  // neighbour marking walk of :494-520 / :538-564 (stops at the cloud boundary, see header)
  auto mark_neighbours = [&](int ind) {
    for (int l = 1; l <= 5; ++l) {
      if (ind + l >= cloudSize) break;
      float ex = lc[ind + l].x - lc[ind + l - 1].x, ey = lc[ind + l].y - lc[ind + l - 1].y,
            ez = lc[ind + l].z - lc[ind + l - 1].z;
      if (D(ex * ex + ey * ey + ez * ez) > 0.05) break;
      picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; --l) {
      if (ind + l < 0) break;
      float ex = lc[ind + l].x - lc[ind + l + 1].x, ey = lc[ind + l].y - lc[ind + l + 1].y,
            ez = lc[ind + l].z - lc[ind + l + 1].z;
      if (D(ex * ex + ey * ey + ez * ez) > 0.05) break;
      picked[ind + l] = 1;
    }
  };

  // :460-582 per ring x 6 segments
  o.sharp.clear(); o.lsharp.clear(); o.flat.clear(); o.lflat.clear();
  std::vector<P> lessFlatScan, lessFlatScanDS;
  for (int i = 0; i < N; ++i) {
    lessFlatScan.clear();
    for (int j = 0; j < 6; ++j) {
      int sp = (startInd[i] * (6 - j) + endInd[i] * j) / 6;
      int ep = (startInd[i] * (5 - j) + endInd[i] * (j + 1)) / 6 - 1;
      if (sp < 0 || ep >= cloudSize) continue;  // out-of-cloud ranges: undefined in the reference
      // :466-474 O(n^2) stable insertion sort by curvature (no early exit, as the reference)
      for (int k = sp + 1; k <= ep; ++k)
        for (int l = k; l >= sp + 1; --l)
          if (curv[sortInd[l]] < curv[sortInd[l - 1]]) std::swap(sortInd[l - 1], sortInd[l]);
      // :476-522 sharp / less sharp
      int largestPickedNum = 0;
      for (int k = ep; k >= sp; --k) {
        int ind = sortInd[k];
        if (picked[ind] == 0 && D(curv[ind]) > 0.1) {
          largestPickedNum++;
          if (largestPickedNum <= 2) {
            label[ind] = 2;
            o.sharp.push_back(lc[ind]);
            o.lsharp.push_back(lc[ind]);
          } else if (largestPickedNum <= 20) {
            label[ind] = 1;
            o.lsharp.push_back(lc[ind]);
          } else {
            break;
          }
          picked[ind] = 1;
          mark_neighbours(ind);
        }
      }
      // :524-566 flat (break after the 4th push, before marking: Q7)
      int smallestPickedNum = 0;
      for (int k = sp; k <= ep; ++k) {
        int ind = sortInd[k];
        if (picked[ind] == 0 && D(curv[ind]) < 0.1) {
          label[ind] = -1;
          o.flat.push_back(lc[ind]);
          smallestPickedNum++;
          if (smallestPickedNum >= 4) break;
          picked[ind] = 1;
          mark_neighbours(ind);
        }
      }
      // :568-572
      for (int k = sp; k <= ep; ++k)
        if (label[k] <= 0) lessFlatScan.push_back(lc[k]);
    }
    // :575-581
    voxel_grid(lessFlatScan, 0.2f, lessFlatScanDS);
    o.lflat.insert(o.lflat.end(), lessFlatScanDS.begin(), lessFlatScanDS.end());
  }
  return LOAM_OK;
}

// ===================================================================== odometry
struct OdState {
  bool inited = false;
  float transform[6] = {0, 0, 0, 0, 0, 0};
  float transformSum[6] = {0, 0, 0, 0, 0, 0};
  std::vector<P> cornerLast, surfLast;
  KdTree kdCorner, kdSurf;
  int cornerLastNum = 0, surfLastNum = 0;  // globals, zero-initialised (Q8)
  bool isDegenerate = false;
  float matP[36] = {0};
  int frameCount = 1;                       // = skipFrameNum (:407)
  // imu_trans (/imu_trans) values; zero without IMU
  float imuRollStart = 0, imuPitchStart = 0, imuYawStart = 0;
  float imuRollLast = 0, imuPitchLast = 0, imuYawLast = 0;
  float imuShiftFromStartX = 0, imuShiftFromStartY = 0, imuShiftFromStartZ = 0;
  float imuVeloFromStartX = 0, imuVeloFromStartY = 0, imuVeloFromStartZ = 0;
  // stats
  uint64_t iters = 0, assoc = 0, rows_sum = 0, queries = 0;
  uint64_t deg_steps = 0, nan_skips = 0;  // updates through the degeneracy projection / NaN guard
};

// :101-124
void transform_to_start(const OdState& s, const P& pi, P& po) {
  const float* t = s.transform;
  float sc = 10 * (pi.intensity - (int)pi.intensity);
  float rx = sc * t[0], ry = sc * t[1], rz = sc * t[2];
  float tx = sc * t[3], ty = sc * t[4], tz = sc * t[5];
  float x1 = (float)(dcos(rz) * D(pi.x - tx) + dsin(rz) * D(pi.y - ty));
  float y1 = (float)(-dsin(rz) * D(pi.x - tx) + dcos(rz) * D(pi.y - ty));
  float z1 = (pi.z - tz);
  float x2 = x1;
  float y2 = (float)(dcos(rx) * D(y1) + dsin(rx) * D(z1));
  float z2 = (float)(-dsin(rx) * D(y1) + dcos(rx) * D(z1));
  po.x = (float)(dcos(ry) * D(x2) - dsin(ry) * D(z2));
  po.y = y2;
  po.z = (float)(dsin(ry) * D(x2) + dcos(ry) * D(z2));
  po.intensity = pi.intensity;
}

// :126-194
void transform_to_end(const OdState& s, const P& pi, P& po) {
  const float* t = s.transform;
  float sc = 10 * (pi.intensity - (int)pi.intensity);
  float rx = sc * t[0], ry = sc * t[1], rz = sc * t[2];
  float tx = sc * t[3], ty = sc * t[4], tz = sc * t[5];
  float x1 = (float)(dcos(rz) * D(pi.x - tx) + dsin(rz) * D(pi.y - ty));
  float y1 = (float)(-dsin(rz) * D(pi.x - tx) + dcos(rz) * D(pi.y - ty));
  float z1 = (pi.z - tz);
  float x2 = x1;
  float y2 = (float)(dcos(rx) * D(y1) + dsin(rx) * D(z1));
  float z2 = (float)(-dsin(rx) * D(y1) + dcos(rx) * D(z1));
  float x3 = (float)(dcos(ry) * D(x2) - dsin(ry) * D(z2));
  float y3 = y2;
  float z3 = (float)(dsin(ry) * D(x2) + dcos(ry) * D(z2));
  rx = t[0]; ry = t[1]; rz = t[2]; tx = t[3]; ty = t[4]; tz = t[5];
  float x4 = (float)(dcos(ry) * D(x3) + dsin(ry) * D(z3));
  float y4 = y3;
  float z4 = (float)(-dsin(ry) * D(x3) + dcos(ry) * D(z3));
  float x5 = x4;
  float y5 = (float)(dcos(rx) * D(y4) - dsin(rx) * D(z4));
  float z5 = (float)(dsin(rx) * D(y4) + dcos(rx) * D(z4));
  float x6 = (float)(dcos(rz) * D(x5) - dsin(rz) * D(y5) + D(tx));
  float y6 = (float)(dsin(rz) * D(x5) + dcos(rz) * D(y5) + D(ty));
  float z6 = z5 + tz;
  float x7 = (float)(dcos(s.imuRollStart) * D(x6 - s.imuShiftFromStartX) -
                     dsin(s.imuRollStart) * D(y6 - s.imuShiftFromStartY));
  float y7 = (float)(dsin(s.imuRollStart) * D(x6 - s.imuShiftFromStartX) +
                     dcos(s.imuRollStart) * D(y6 - s.imuShiftFromStartY));
  float z7 = z6 - s.imuShiftFromStartZ;
  float x8 = x7;
  float y8 = (float)(dcos(s.imuPitchStart) * D(y7) - dsin(s.imuPitchStart) * D(z7));
  float z8 = (float)(dsin(s.imuPitchStart) * D(y7) + dcos(s.imuPitchStart) * D(z7));
  float x9 = (float)(dcos(s.imuYawStart) * D(x8) + dsin(s.imuYawStart) * D(z8));
  float y9 = y8;
  float z9 = (float)(-dsin(s.imuYawStart) * D(x8) + dcos(s.imuYawStart) * D(z8));
  float x10 = (float)(dcos(s.imuYawLast) * D(x9) - dsin(s.imuYawLast) * D(z9));
  float y10 = y9;
  float z10 = (float)(dsin(s.imuYawLast) * D(x9) + dcos(s.imuYawLast) * D(z9));
  float x11 = x10;
  float y11 = (float)(dcos(s.imuPitchLast) * D(y10) + dsin(s.imuPitchLast) * D(z10));
  float z11 = (float)(-dsin(s.imuPitchLast) * D(y10) + dcos(s.imuPitchLast) * D(z10));
  float ox = (float)(dcos(s.imuRollLast) * D(x11) + dsin(s.imuRollLast) * D(y11));
  float oy = (float)(-dsin(s.imuRollLast) * D(x11) + dcos(s.imuRollLast) * D(y11));
  float oi = (float)(int)pi.intensity;
  po.x = ox; po.y = oy; po.z = z11; po.intensity = oi;
}

// :196-254 (float variables, C double trig)
void plugin_imu_rotation(float bcx, float bcy, float bcz, float blx, float bly, float blz,
                         float alx, float aly, float alz, float& acx, float& acy, float& acz) {
  float sbcx = (float)dsin(bcx), cbcx = (float)dcos(bcx), sbcy = (float)dsin(bcy),
        cbcy = (float)dcos(bcy), sbcz = (float)dsin(bcz), cbcz = (float)dcos(bcz);
  float sblx = (float)dsin(blx), cblx = (float)dcos(blx), sbly = (float)dsin(bly),
        cbly = (float)dcos(bly), sblz = (float)dsin(blz), cblz = (float)dcos(blz);
  float salx = (float)dsin(alx), calx = (float)dcos(alx), saly = (float)dsin(aly),
        caly = (float)dcos(aly), salz = (float)dsin(alz), calz = (float)dcos(alz);
  float srx = -sbcx * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly) -
              cbcx * cbcz *
                  (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                   calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
              cbcx * sbcz *
                  (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                   calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz);
  acx = (float)(-std::asin(D(srx)));
  float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) *
                     (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                      calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                 (cbcy * cbcz + sbcx * sbcy * sbcz) *
                     (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                      calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) +
                 cbcx * sbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) *
                     (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                      calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) -
                 (sbcy * sbcz + cbcy * cbcz * sbcx) *
                     (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                      calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) +
                 cbcx * cbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  acy = (float)std::atan2(D(srycrx) / dcos(acx), D(crycrx) / dcos(acx));
  float srzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) -
                         cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                 cbcx * cbcz *
                     ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) +
                      (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) -
                      calx * cblx * cblz * salz) +
                 cbcx * sbcz *
                     ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                      (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                      calx * cblx * salz * sblz);
  float crzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) -
                         cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                 cbcx * cbcz *
                     ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                      (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                      calx * calz * cblx * cblz) -
                 cbcx * sbcz *
                     ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) +
                      (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) -
                      calx * calz * cblx * sblz);
  acz = (float)std::atan2(D(srzcrx) / dcos(acx), D(crzcrx) / dcos(acx));
}

// :256-273 (double expressions of float arguments)
void accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz, float& ox,
                         float& oy, float& oz) {
  float srx = (float)(dcos(lx) * dcos(cx) * dsin(ly) * dsin(cz) - dcos(cx) * dcos(cz) * dsin(lx) -
                      dcos(lx) * dcos(ly) * dsin(cx));
  ox = (float)(-std::asin(D(srx)));
  float srycrx = (float)(dsin(lx) * (dcos(cy) * dsin(cz) - dcos(cz) * dsin(cx) * dsin(cy)) +
                         dcos(lx) * dsin(ly) * (dcos(cy) * dcos(cz) + dsin(cx) * dsin(cy) * dsin(cz)) +
                         dcos(lx) * dcos(ly) * dcos(cx) * dsin(cy));
  float crycrx = (float)(dcos(lx) * dcos(ly) * dcos(cx) * dcos(cy) -
                         dcos(lx) * dsin(ly) * (dcos(cz) * dsin(cy) - dcos(cy) * dsin(cx) * dsin(cz)) -
                         dsin(lx) * (dsin(cy) * dsin(cz) + dcos(cy) * dcos(cz) * dsin(cx)));
  oy = (float)std::atan2(D(srycrx) / dcos(ox), D(crycrx) / dcos(ox));
  float srzcrx = (float)(dsin(cx) * (dcos(lz) * dsin(ly) - dcos(ly) * dsin(lx) * dsin(lz)) +
                         dcos(cx) * dsin(cz) * (dcos(ly) * dcos(lz) + dsin(lx) * dsin(ly) * dsin(lz)) +
                         dcos(lx) * dcos(cx) * dcos(cz) * dsin(lz));
  float crzcrx = (float)(dcos(lx) * dcos(lz) * dcos(cx) * dcos(cz) -
                         dcos(cx) * dsin(cz) * (dcos(ly) * dsin(lz) - dcos(lz) * dsin(lx) * dsin(ly)) -
                         dsin(cx) * (dsin(ly) * dsin(lz) + dcos(ly) * dcos(lz) * dsin(lx)));
  oz = (float)std::atan2(D(srzcrx) / dcos(ox), D(crzcrx) / dcos(ox));
}

// the L-M step shared by odometry (:765-826) and mapping (:922-974): AtA/AtB (double-accumulated
// gemm), QR solve, iteration-0 degeneracy projection.  Returns matX.
void lm_solve(const std::vector<float>& A, const std::vector<float>& B, int rows, int iter,
              float eig_thresh, bool& isDegenerate, float* matP, float* X) {
  std::vector<float> At((size_t)6 * rows);
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < 6; ++j) At[(size_t)j * rows + i] = A[(size_t)i * 6 + j];
  float AtA[36], AtB[6];
  gemm_d(At.data(), A.data(), 6, rows, 6, AtA);
  gemm_d(At.data(), B.data(), 6, rows, 1, AtB);
  qr_solve(AtA, AtB, 6, 6, X);
  if (iter == 0) {
    float E[6], V[36], V2[36], Vi[36];
    jacobi(AtA, 6, E, V);
    std::memcpy(V2, V, sizeof(V));
    isDegenerate = false;
    for (int i = 5; i >= 0; --i) {
      if (E[i] < eig_thresh) {
        for (int j = 0; j < 6; ++j) V2[i * 6 + j] = 0;
        isDegenerate = true;
      } else {
        break;
      }
    }
    lu_inv(V, 6, Vi);
    gemm_d(Vi, V2, 6, 6, 6, matP);
  }
  if (isDegenerate) {
    float X2[6];
    std::memcpy(X2, X, sizeof(X2));
    gemm_d(matP, X2, 6, 6, 1, X);
  }
}

inline float delta_r(const float* X) {
  return (float)std::sqrt(std::pow(rad2deg(D(X[0])), 2) + std::pow(rad2deg(D(X[1])), 2) +
                          std::pow(rad2deg(D(X[2])), 2));
}
inline float delta_t(const float* X) {
  return (float)std::sqrt(std::pow(D(X[3] * 100), 2) + std::pow(D(X[4] * 100), 2) +
                          std::pow(D(X[5] * 100), 2));
}

struct OdIn {
  const std::vector<P>* sharp; const std::vector<P>* lsharp; const std::vector<P>* flat;
  const std::vector<P>* lflat; const std::vector<P>* full;
};
struct OdOut {
  float sum[6];
  std::vector<P> cornerLast, surfLast, full;
  int published = 0;
};

// the L-M of :465-828
void od_lm(const Cfg& cfg, OdState& s, const std::vector<P>& sharp, const std::vector<P>& flat) {
  float* transform = s.transform;
  const int cornerPointsSharpNum = (int)sharp.size();
  const int surfPointsFlatNum = (int)flat.size();
  std::vector<float> ind1c(cornerPointsSharpNum, -1), ind2c(cornerPointsSharpNum, -1);
  std::vector<float> ind1s(surfPointsFlatNum, -1), ind2s(surfPointsFlatNum, -1),
      ind3s(surfPointsFlatNum, -1);
  std::vector<P> cloudOri, coeffSel;  // cleared once per frame (:458-459): rows accumulate (Q12)
  std::vector<int> nanIdx;
  int nnI[2];  // k = 1 results (one spare slot keeps -Warray-bounds provable)
  float nnD[2];
  const std::vector<P>& CL = s.cornerLast;
  const std::vector<P>& SL = s.surfLast;
  for (int iterCount = 0; iterCount < cfg.od_max_iter; ++iterCount) {
    s.iters++;
    if (iterCount % 5 == 0) s.assoc++;
    for (int i = 0; i < cornerPointsSharpNum; ++i) {
      P pointSel;
      transform_to_start(s, sharp[i], pointSel);
      if (iterCount % 5 == 0) {
        s.queries++;
        // :476 removeNaNFromPointCloud on the dense CornerLast: an O(C) index fill per query
        nanIdx.resize(CL.size());
        std::iota(nanIdx.begin(), nanIdx.end(), 0);
        int closestPointInd = -1, minPointInd2 = -1;
        int got = s.kdCorner.knn(pointSel.x, pointSel.y, pointSel.z, 1, nnI, nnD);
        if (got > 0 && D(nnD[0]) < 25) {
          closestPointInd = nnI[0];
          int closestPointScan = (int)CL[closestPointInd].intensity;
          float minPointSqDis2 = 25;
          // Q11: the reference bounds the forward window by this sweep's cornerPointsSharpNum
          // (:486), reading past CornerLast when that exceeds it (UB).  Defined here, as in the
          // engine (od.hip k_od_assoc), as min(cornerPointsSharpNum, |CornerLast|).
          const int fwdEnd = std::min(cornerPointsSharpNum, (int)CL.size());
          for (int j = closestPointInd + 1; j < fwdEnd; ++j) {
            if (D((int)CL[j].intensity) > closestPointScan + 2.5) break;
            float pointSqDis = (CL[j].x - pointSel.x) * (CL[j].x - pointSel.x) +
                               (CL[j].y - pointSel.y) * (CL[j].y - pointSel.y) +
                               (CL[j].z - pointSel.z) * (CL[j].z - pointSel.z);
            if ((int)CL[j].intensity > closestPointScan && pointSqDis < minPointSqDis2) {
              minPointSqDis2 = pointSqDis;
              minPointInd2 = j;
            }
          }
          for (int j = closestPointInd - 1; j >= 0; --j) {
            if (D((int)CL[j].intensity) < closestPointScan - 2.5) break;
            float pointSqDis = (CL[j].x - pointSel.x) * (CL[j].x - pointSel.x) +
                               (CL[j].y - pointSel.y) * (CL[j].y - pointSel.y) +
                               (CL[j].z - pointSel.z) * (CL[j].z - pointSel.z);
            if ((int)CL[j].intensity < closestPointScan && pointSqDis < minPointSqDis2) {
              minPointSqDis2 = pointSqDis;
              minPointInd2 = j;
            }
          }
        }
        ind1c[i] = (float)closestPointInd;
        ind2c[i] = (float)minPointInd2;
      }
      if (ind2c[i] >= 0) {  // :530-583
        const P& t1 = CL[(int)ind1c[i]];
        const P& t2 = CL[(int)ind2c[i]];
        float x0 = pointSel.x, y0 = pointSel.y, z0 = pointSel.z;
        float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
        float a012 = (float)std::sqrt(D(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) *
                                            ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                                        ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) *
                                            ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                                        ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) *
                                            ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))));
        float l12 = (float)std::sqrt(D((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) +
                                       (z1 - z2) * (z1 - z2)));
        float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                    (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) /
                   a012 / l12;
        float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                     (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) /
                   a012 / l12;
        float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                     (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) /
                   a012 / l12;
        float ld2 = a012 / l12;
        float sw = 1;
        if (iterCount >= 5) sw = (float)(1 - 1.8 * std::fabs(D(ld2)));
        P coeff{sw * la, sw * lb, sw * lc, sw * ld2};
        if (D(sw) > 0.1 && ld2 != 0) {
          cloudOri.push_back(sharp[i]);
          coeffSel.push_back(coeff);
        }
      }
    }
    for (int i = 0; i < surfPointsFlatNum; ++i) {
      P pointSel;
      transform_to_start(s, flat[i], pointSel);
      if (iterCount % 5 == 0) {
        s.queries++;
        int got = s.kdSurf.knn(pointSel.x, pointSel.y, pointSel.z, 1, nnI, nnD);
        int closestPointInd = -1, minPointInd2 = -1, minPointInd3 = -1;
        if (got > 0 && D(nnD[0]) < 25) {
          closestPointInd = nnI[0];
          int closestPointScan = (int)SL[closestPointInd].intensity;
          float minPointSqDis2 = 25, minPointSqDis3 = 25;
          // Q11 (:598): same clamp, min(surfPointsFlatNum, |SurfLast|)
          const int fwdEnd = std::min(surfPointsFlatNum, (int)SL.size());
          for (int j = closestPointInd + 1; j < fwdEnd; ++j) {
            if (D((int)SL[j].intensity) > closestPointScan + 2.5) break;
            float pointSqDis = (SL[j].x - pointSel.x) * (SL[j].x - pointSel.x) +
                               (SL[j].y - pointSel.y) * (SL[j].y - pointSel.y) +
                               (SL[j].z - pointSel.z) * (SL[j].z - pointSel.z);
            if ((int)SL[j].intensity <= closestPointScan) {
              if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
            } else {
              if (pointSqDis < minPointSqDis3) { minPointSqDis3 = pointSqDis; minPointInd3 = j; }
            }
          }
          for (int j = closestPointInd - 1; j >= 0; --j) {
            if (D((int)SL[j].intensity) < closestPointScan - 2.5) break;
            float pointSqDis = (SL[j].x - pointSel.x) * (SL[j].x - pointSel.x) +
                               (SL[j].y - pointSel.y) * (SL[j].y - pointSel.y) +
                               (SL[j].z - pointSel.z) * (SL[j].z - pointSel.z);
            if ((int)SL[j].intensity >= closestPointScan) {
              if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
            } else {
              if (pointSqDis < minPointSqDis3) { minPointSqDis3 = pointSqDis; minPointInd3 = j; }
            }
          }
        }
        ind1s[i] = (float)closestPointInd;
        ind2s[i] = (float)minPointInd2;
        ind3s[i] = (float)minPointInd3;
      }
      if (ind2s[i] >= 0 && ind3s[i] >= 0) {  // :653-694
        const P& t1 = SL[(int)ind1s[i]];
        const P& t2 = SL[(int)ind2s[i]];
        const P& t3 = SL[(int)ind3s[i]];
        float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
        float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
        float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
        float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
        float ps = (float)std::sqrt(D(pa * pa + pb * pb + pc * pc));
        pa /= ps; pb /= ps; pc /= ps; pd /= ps;
        float pd2 = pa * pointSel.x + pb * pointSel.y + pc * pointSel.z + pd;
        float sw = 1;
        if (iterCount >= 5)
          sw = (float)(1 - 1.8 * std::fabs(D(pd2)) /
                               std::sqrt(std::sqrt(D(pointSel.x * pointSel.x + pointSel.y * pointSel.y +
                                                     pointSel.z * pointSel.z))));
        P coeff{sw * pa, sw * pb, sw * pc, sw * pd2};
        if (D(sw) > 0.1 && pd2 != 0) {
          cloudOri.push_back(flat[i]);
          coeffSel.push_back(coeff);
        }
      }
    }
    const int pointSelNum = (int)cloudOri.size();
    s.rows_sum += (uint64_t)pointSelNum;
    if (pointSelNum < 10) continue;
    // :702-764 J rows at the current transform (recomputed for every accumulated row)
    std::vector<float> A((size_t)pointSelNum * 6), B(pointSelNum);
    for (int i = 0; i < pointSelNum; ++i) {
      const P& po = cloudOri[i];
      const P& cf = coeffSel[i];
      float sw = 1;
      float srx = (float)dsin(sw * transform[0]), crx = (float)dcos(sw * transform[0]);
      float sry = (float)dsin(sw * transform[1]), cry = (float)dcos(sw * transform[1]);
      float srz = (float)dsin(sw * transform[2]), crz = (float)dcos(sw * transform[2]);
      float tx = sw * transform[3], ty = sw * transform[4], tz = sw * transform[5];
      float arx = (-sw * crx * sry * srz * po.x + sw * crx * crz * sry * po.y + sw * srx * sry * po.z +
                   sw * tx * crx * sry * srz - sw * ty * crx * crz * sry - sw * tz * srx * sry) * cf.x +
                  (sw * srx * srz * po.x - sw * crz * srx * po.y + sw * crx * po.z +
                   sw * ty * crz * srx - sw * tz * crx - sw * tx * srx * srz) * cf.y +
                  (sw * crx * cry * srz * po.x - sw * crx * cry * crz * po.y - sw * cry * srx * po.z +
                   sw * tz * cry * srx + sw * ty * crx * cry * crz - sw * tx * crx * cry * srz) * cf.z;
      float ary = ((-sw * crz * sry - sw * cry * srx * srz) * po.x +
                   (sw * cry * crz * srx - sw * sry * srz) * po.y - sw * crx * cry * po.z +
                   tx * (sw * crz * sry + sw * cry * srx * srz) +
                   ty * (sw * sry * srz - sw * cry * crz * srx) + sw * tz * crx * cry) * cf.x +
                  ((sw * cry * crz - sw * srx * sry * srz) * po.x +
                   (sw * cry * srz + sw * crz * srx * sry) * po.y - sw * crx * sry * po.z +
                   sw * tz * crx * sry - ty * (sw * cry * srz + sw * crz * srx * sry) -
                   tx * (sw * cry * crz - sw * srx * sry * srz)) * cf.z;
      float arz = ((-sw * cry * srz - sw * crz * srx * sry) * po.x +
                   (sw * cry * crz - sw * srx * sry * srz) * po.y +
                   tx * (sw * cry * srz + sw * crz * srx * sry) -
                   ty * (sw * cry * crz - sw * srx * sry * srz)) * cf.x +
                  (-sw * crx * crz * po.x - sw * crx * srz * po.y + sw * ty * crx * srz +
                   sw * tx * crx * crz) * cf.y +
                  ((sw * cry * crz * srx - sw * sry * srz) * po.x +
                   (sw * crz * sry + sw * cry * srx * srz) * po.y +
                   tx * (sw * sry * srz - sw * cry * crz * srx) -
                   ty * (sw * crz * sry + sw * cry * srx * srz)) * cf.z;
      float atx = -sw * (cry * crz - srx * sry * srz) * cf.x + sw * crx * srz * cf.y -
                  sw * (crz * sry + cry * srx * srz) * cf.z;
      float aty = -sw * (cry * srz + crz * srx * sry) * cf.x - sw * crx * crz * cf.y -
                  sw * (sry * srz - cry * crz * srx) * cf.z;
      float atz = sw * crx * sry * cf.x - sw * srx * cf.y - sw * crx * cry * cf.z;
      float d2 = cf.intensity;
      float* a = &A[(size_t)i * 6];
      a[0] = arx; a[1] = ary; a[2] = arz; a[3] = atx; a[4] = aty; a[5] = atz;
      B[i] = (float)(-0.05 * D(d2));
    }
    float X[6];
    lm_solve(A, B, pointSelNum, iterCount, 10.0f, s.isDegenerate, s.matP, X);
    if (s.isDegenerate) s.deg_steps++;
    bool nan = std::isnan(X[0]) || std::isnan(X[1]) || std::isnan(X[2]) || std::isnan(X[3]) ||
               std::isnan(X[4]) || std::isnan(X[5]);
    if (!nan)  // :799-811 NaN guard (Q16)
      for (int q = 0; q < 6; ++q) transform[q] += X[q];
    else
      s.nan_skips++;
    float deltaR = delta_r(X), deltaT = delta_t(X);
    if (D(deltaR) < 0.1 && D(deltaT) < 0.1) break;
  }
}

// laserOdometry loop body :420-931
// hook of the oracle's own tests (oracle_problem_with_od): the odometry L-M solution replaced by a
// given transform before the pose accumulation and TransformToEnd
thread_local const float* g_od_override = nullptr;

void od_body(const Cfg& cfg, OdState& s, const OdIn& in, OdOut& out) {
  out.published = 0;
  if (!s.inited) {  // :427-456
    s.cornerLast = *in.lsharp;
    s.surfLast = *in.lflat;
    s.kdCorner.build(s.cornerLast);
    s.kdSurf.build(s.surfLast);
    out.cornerLast = s.cornerLast;
    out.surfLast = s.surfLast;
    out.published = LOAM_PUB_CLOUDS;
    s.transformSum[0] += s.imuPitchStart;
    s.transformSum[2] += s.imuRollStart;
    s.inited = true;
    return;
  }
  const float scanPeriod = 0.1f;  // const float in laserOdometry.cpp:49
  s.transform[3] -= s.imuVeloFromStartX * scanPeriod;
  s.transform[4] -= s.imuVeloFromStartY * scanPeriod;
  s.transform[5] -= s.imuVeloFromStartZ * scanPeriod;
  if (s.cornerLastNum > 10 && s.surfLastNum > 100) od_lm(cfg, s, *in.sharp, *in.flat);
  if (g_od_override)
    for (int k = 0; k < 6; ++k) s.transform[k] = g_od_override[k];

  // :830-856
  float rx, ry, rz;
  accumulate_rotation(s.transformSum[0], s.transformSum[1], s.transformSum[2], -s.transform[0],
                      (float)(-D(s.transform[1]) * 1.05), -s.transform[2], rx, ry, rz);
  float x1 = (float)(dcos(rz) * D(s.transform[3] - s.imuShiftFromStartX) -
                     dsin(rz) * D(s.transform[4] - s.imuShiftFromStartY));
  float y1 = (float)(dsin(rz) * D(s.transform[3] - s.imuShiftFromStartX) +
                     dcos(rz) * D(s.transform[4] - s.imuShiftFromStartY));
  float z1 = (float)(D(s.transform[5]) * 1.05 - D(s.imuShiftFromStartZ));
  float x2 = x1;
  float y2 = (float)(dcos(rx) * D(y1) - dsin(rx) * D(z1));
  float z2 = (float)(dsin(rx) * D(y1) + dcos(rx) * D(z1));
  float tx = (float)(D(s.transformSum[3]) - (dcos(ry) * D(x2) + dsin(ry) * D(z2)));
  float ty = s.transformSum[4] - y2;
  float tz = (float)(D(s.transformSum[5]) - (-dsin(ry) * D(x2) + dcos(ry) * D(z2)));
  plugin_imu_rotation(rx, ry, rz, s.imuPitchStart, s.imuYawStart, s.imuRollStart, s.imuPitchLast,
                      s.imuYawLast, s.imuRollLast, rx, ry, rz);
  s.transformSum[0] = rx; s.transformSum[1] = ry; s.transformSum[2] = rz;
  s.transformSum[3] = tx; s.transformSum[4] = ty; s.transformSum[5] = tz;
  std::memcpy(out.sum, s.transformSum, sizeof(out.sum));
  out.published = LOAM_PUB_POSE;

  // :875-891
  std::vector<P> lsharp(in.lsharp->size()), lflat(in.lflat->size());
  for (size_t i = 0; i < lsharp.size(); ++i) transform_to_end(s, (*in.lsharp)[i], lsharp[i]);
  for (size_t i = 0; i < lflat.size(); ++i) transform_to_end(s, (*in.lflat)[i], lflat[i]);
  s.frameCount++;
  bool pub = s.frameCount >= cfg.skip_frame_num + 1;
  if (pub) {
    out.full.resize(in.full->size());
    for (size_t i = 0; i < out.full.size(); ++i) transform_to_end(s, (*in.full)[i], out.full[i]);
  }
  // :893-908
  s.cornerLast.swap(lsharp);
  s.surfLast.swap(lflat);
  s.cornerLastNum = (int)s.cornerLast.size();
  s.surfLastNum = (int)s.surfLast.size();
  if (s.cornerLastNum > 10 && s.surfLastNum > 100) {
    s.kdCorner.build(s.cornerLast);
    s.kdSurf.build(s.surfLast);
  }
  if (pub) {  // :910-930
    s.frameCount = 0;
    out.cornerLast = s.cornerLast;
    out.surfLast = s.surfLast;
    out.published |= LOAM_PUB_CLOUDS | LOAM_PUB_FULL;
  }
}

// ===================================================================== mapping
const int kW = 21, kH = 11, kDp = 21, kNum = kW * kH * kDp;  // :64-70

struct MpState {
  float transformSum[6] = {0}, transformIncre[6] = {0}, transformTobeMapped[6] = {0};
  float transformBefMapped[6] = {0}, transformAftMapped[6] = {0};
  int cenW = 10, cenH = 5, cenD = 10;
  std::vector<std::vector<P>> corner, surf;
  int frameCount = 0, mapFrameCount = 4;  // stackFrameNum - 1, mapFrameNum - 1 (:404-405)
  bool isDegenerate = false;
  float matP[36] = {0};
  uint64_t iters = 0, rows_sum = 0, stack = 0, map_points = 0, valid_points = 0;
  uint64_t deg_steps = 0, shifts = 0;  // updates through the degeneracy projection / slab shifts
  // laserMapping's IMU queue (:101-108), fed by its imuHandler (:323-335)
  int imuFront = 0, imuLast = -1;
  double imuTime[kImuQue] = {0};
  float imuRoll[kImuQue] = {0}, imuPitch[kImuQue] = {0};
  MpState() : corner(kNum), surf(kNum) {}
};

// :110-197
void transform_associate_to_map(MpState& m) {
  const float* S = m.transformSum;
  const float* B = m.transformBefMapped;
  const float* A = m.transformAftMapped;
  float* I = m.transformIncre;
  float* T = m.transformTobeMapped;
  float x1 = (float)(dcos(S[1]) * D(B[3] - S[3]) - dsin(S[1]) * D(B[5] - S[5]));
  float y1 = B[4] - S[4];
  float z1 = (float)(dsin(S[1]) * D(B[3] - S[3]) + dcos(S[1]) * D(B[5] - S[5]));
  float x2 = x1;
  float y2 = (float)(dcos(S[0]) * D(y1) + dsin(S[0]) * D(z1));
  float z2 = (float)(-dsin(S[0]) * D(y1) + dcos(S[0]) * D(z1));
  I[3] = (float)(dcos(S[2]) * D(x2) + dsin(S[2]) * D(y2));
  I[4] = (float)(-dsin(S[2]) * D(x2) + dcos(S[2]) * D(y2));
  I[5] = z2;
  float sbcx = (float)dsin(S[0]), cbcx = (float)dcos(S[0]), sbcy = (float)dsin(S[1]),
        cbcy = (float)dcos(S[1]), sbcz = (float)dsin(S[2]), cbcz = (float)dcos(S[2]);
  float sblx = (float)dsin(B[0]), cblx = (float)dcos(B[0]), sbly = (float)dsin(B[1]),
        cbly = (float)dcos(B[1]), sblz = (float)dsin(B[2]), cblz = (float)dcos(B[2]);
  float salx = (float)dsin(A[0]), calx = (float)dcos(A[0]), saly = (float)dsin(A[1]),
        caly = (float)dcos(A[1]), salz = (float)dsin(A[2]), calz = (float)dcos(A[2]);
  float srx = -sbcx * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly) -
              cbcx * cbcz *
                  (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                   calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
              cbcx * sbcz *
                  (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                   calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz);
  T[0] = (float)(-std::asin(D(srx)));
  float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) *
                     (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                      calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                 (cbcy * cbcz + sbcx * sbcy * sbcz) *
                     (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                      calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) +
                 cbcx * sbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) *
                     (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                      calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) -
                 (sbcy * sbcz + cbcy * cbcz * sbcx) *
                     (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                      calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) +
                 cbcx * cbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  T[1] = (float)std::atan2(D(srycrx) / dcos(T[0]), D(crycrx) / dcos(T[0]));
  float srzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) -
                         cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                 cbcx * cbcz *
                     ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) +
                      (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) -
                      calx * cblx * cblz * salz) +
                 cbcx * sbcz *
                     ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                      (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                      calx * cblx * salz * sblz);
  float crzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) -
                         cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                 cbcx * cbcz *
                     ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                      (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                      calx * calz * cblx * cblz) -
                 cbcx * sbcz *
                     ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) +
                      (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) -
                      calx * calz * cblx * sblz);
  T[2] = (float)std::atan2(D(srzcrx) / dcos(T[0]), D(crzcrx) / dcos(T[0]));
  x1 = (float)(dcos(T[2]) * D(I[3]) - dsin(T[2]) * D(I[4]));
  y1 = (float)(dsin(T[2]) * D(I[3]) + dcos(T[2]) * D(I[4]));
  z1 = I[5];
  x2 = x1;
  y2 = (float)(dcos(T[0]) * D(y1) - dsin(T[0]) * D(z1));
  z2 = (float)(dsin(T[0]) * D(y1) + dcos(T[0]) * D(z1));
  T[3] = (float)(D(A[3]) - (dcos(T[1]) * D(x2) + dsin(T[1]) * D(z2)));
  T[4] = A[4] - y2;
  T[5] = (float)(D(A[5]) - (-dsin(T[1]) * D(x2) + dcos(T[1]) * D(z2)));
}

// :234-252
inline void point_associate_to_map(const float* T, const P& pi, P& po) {
  float x1 = (float)(dcos(T[2]) * D(pi.x) - dsin(T[2]) * D(pi.y));
  float y1 = (float)(dsin(T[2]) * D(pi.x) + dcos(T[2]) * D(pi.y));
  float z1 = pi.z;
  float x2 = x1;
  float y2 = (float)(dcos(T[0]) * D(y1) - dsin(T[0]) * D(z1));
  float z2 = (float)(dsin(T[0]) * D(y1) + dcos(T[0]) * D(z1));
  float ox = (float)(dcos(T[1]) * D(x2) + dsin(T[1]) * D(z2) + D(T[3]));
  float oy = y2 + T[4];
  float oz = (float)(-dsin(T[1]) * D(x2) + dcos(T[1]) * D(z2) + D(T[5]));
  float oi = pi.intensity;
  po.x = ox; po.y = oy; po.z = oz; po.intensity = oi;
}

// :254-272
inline void point_associate_tobe_mapped(const float* T, const P& pi, P& po) {
  float x1 = (float)(dcos(T[1]) * D(pi.x - T[3]) - dsin(T[1]) * D(pi.z - T[5]));
  float y1 = pi.y - T[4];
  float z1 = (float)(dsin(T[1]) * D(pi.x - T[3]) + dcos(T[1]) * D(pi.z - T[5]));
  float x2 = x1;
  float y2 = (float)(dcos(T[0]) * D(y1) + dsin(T[0]) * D(z1));
  float z2 = (float)(-dsin(T[0]) * D(y1) + dcos(T[0]) * D(z1));
  float ox = (float)(dcos(T[2]) * D(x2) + dsin(T[2]) * D(y2));
  float oy = (float)(-dsin(T[2]) * D(x2) + dcos(T[2]) * D(y2));
  float oi = pi.intensity;
  po.x = ox; po.y = oy; po.z = z2; po.intensity = oi;
}

inline int cube_of(float v, int cen) {  // :446-452, :983-989
  int c = (int)((D(v) + 25.0) / 50.0) + cen;
  if (D(v) + 25.0 < 0) c--;
  return c;
}

// the grid recentring of :454-614: shift whole slabs, the cleared cube moves to the other end
void shift_axis(MpState& m, int axis, int dir) {
  const int dims[3] = {kW, kH, kDp};
  const int n = dims[axis];
  auto at = [&](int a, int b, int c) -> int {  // (i, j, k) with the axis coordinate = c
    int i = 0, j = 0, k = 0;
    if (axis == 0) { i = c; j = a; k = b; }
    else if (axis == 1) { i = a; j = c; k = b; }
    else { i = a; j = b; k = c; }
    return i + kW * j + kW * kH * k;
  };
  const int na = axis == 0 ? kH : kW;
  const int nb = axis == 2 ? kH : kDp;
  for (int a = 0; a < na; ++a)
    for (int b = 0; b < nb; ++b) {
      if (dir > 0) {  // centre index < 3: move toward higher index, last slot wraps to 0
        std::vector<P> tc = std::move(m.corner[at(a, b, n - 1)]);
        std::vector<P> ts = std::move(m.surf[at(a, b, n - 1)]);
        for (int c = n - 1; c >= 1; --c) {
          m.corner[at(a, b, c)] = std::move(m.corner[at(a, b, c - 1)]);
          m.surf[at(a, b, c)] = std::move(m.surf[at(a, b, c - 1)]);
        }
        tc.clear(); ts.clear();
        m.corner[at(a, b, 0)] = std::move(tc);
        m.surf[at(a, b, 0)] = std::move(ts);
      } else {
        std::vector<P> tc = std::move(m.corner[at(a, b, 0)]);
        std::vector<P> ts = std::move(m.surf[at(a, b, 0)]);
        for (int c = 0; c < n - 1; ++c) {
          m.corner[at(a, b, c)] = std::move(m.corner[at(a, b, c + 1)]);
          m.surf[at(a, b, c)] = std::move(m.surf[at(a, b, c + 1)]);
        }
        tc.clear(); ts.clear();
        m.corner[at(a, b, n - 1)] = std::move(tc);
        m.surf[at(a, b, n - 1)] = std::move(ts);
      }
    }
}

struct MpOut { float aft[6], bef[6]; std::vector<P> registered, surround; bool surround_pub = false; };

// laserMapping loop body :420-1094 (stackFrameNum = 1: every synchronised frame is processed)
void mp_body(const Cfg& cfg, MpState& m, const std::vector<P>& cornerLast,
             const std::vector<P>& surfLast, const std::vector<P>& full, MpOut& out,
             double timeLaserOdometry = 0.0) {
  float* T = m.transformTobeMapped;
  std::vector<P> cornerStack2, surfStack2;
  m.frameCount++;
  // :421-435
  transform_associate_to_map(m);
  cornerStack2.resize(cornerLast.size());
  for (size_t i = 0; i < cornerLast.size(); ++i) point_associate_to_map(T, cornerLast[i], cornerStack2[i]);
  surfStack2.resize(surfLast.size());
  for (size_t i = 0; i < surfLast.size(); ++i) point_associate_to_map(T, surfLast[i], surfStack2[i]);
  m.frameCount = 0;

  // :440-452
  P onY{0.0f, 10.0f, 0.0f, 0.0f};
  point_associate_to_map(T, onY, onY);
  int cI = cube_of(T[3], m.cenW), cJ = cube_of(T[4], m.cenH), cK = cube_of(T[5], m.cenD);
  // :454-614
  while (cI < 3) { shift_axis(m, 0, +1); cI++; m.cenW++; m.shifts++; }
  while (cI >= kW - 3) { shift_axis(m, 0, -1); cI--; m.cenW--; m.shifts++; }
  while (cJ < 3) { shift_axis(m, 1, +1); cJ++; m.cenH++; m.shifts++; }
  while (cJ >= kH - 3) { shift_axis(m, 1, -1); cJ--; m.cenH--; m.shifts++; }
  while (cK < 3) { shift_axis(m, 2, +1); cK++; m.cenD++; m.shifts++; }
  while (cK >= kDp - 3) { shift_axis(m, 2, -1); cK--; m.cenD--; m.shifts++; }

  // :616-672 FOV cube selection
  std::vector<int> valid, surround;
  for (int i = cI - 2; i <= cI + 2; ++i)
    for (int j = cJ - 2; j <= cJ + 2; ++j)
      for (int k = cK - 2; k <= cK + 2; ++k) {
        if (!(i >= 0 && i < kW && j >= 0 && j < kH && k >= 0 && k < kDp)) continue;
        float centerX = (float)(50.0 * (i - m.cenW));
        float centerY = (float)(50.0 * (j - m.cenH));
        float centerZ = (float)(50.0 * (k - m.cenD));
        bool inFOV = false;
        for (int ii = -1; ii <= 1; ii += 2)
          for (int jj = -1; jj <= 1; jj += 2)
            for (int kk = -1; kk <= 1; kk += 2) {
              float cornerX = (float)(D(centerX) + 25.0 * ii);
              float cornerY = (float)(D(centerY) + 25.0 * jj);
              float cornerZ = (float)(D(centerZ) + 25.0 * kk);
              float sq1 = (T[3] - cornerX) * (T[3] - cornerX) + (T[4] - cornerY) * (T[4] - cornerY) +
                          (T[5] - cornerZ) * (T[5] - cornerZ);
              float sq2 = (onY.x - cornerX) * (onY.x - cornerX) + (onY.y - cornerY) * (onY.y - cornerY) +
                          (onY.z - cornerZ) * (onY.z - cornerZ);
              float check1 = (float)(100.0 + D(sq1) - D(sq2) - 10.0 * std::sqrt(3.0) * std::sqrt(D(sq1)));
              float check2 = (float)(100.0 + D(sq1) - D(sq2) + 10.0 * std::sqrt(3.0) * std::sqrt(D(sq1)));
              if (check1 < 0 && check2 > 0) inFOV = true;
            }
        if (inFOV) valid.push_back(i + kW * j + kW * kH * k);
        surround.push_back(i + kW * j + kW * kH * k);  // laserCloudSurroundInd (:667-669)
      }
  // :674-681
  std::vector<P> cornerFromMap, surfFromMap;
  for (int ind : valid) {
    cornerFromMap.insert(cornerFromMap.end(), m.corner[ind].begin(), m.corner[ind].end());
    surfFromMap.insert(surfFromMap.end(), m.surf[ind].begin(), m.surf[ind].end());
  }
  const int cornerFromMapNum = (int)cornerFromMap.size(), surfFromMapNum = (int)surfFromMap.size();
  m.map_points += (uint64_t)(cornerFromMapNum + surfFromMapNum);
  // :683-704
  for (auto& p : cornerStack2) point_associate_tobe_mapped(T, p, p);
  for (auto& p : surfStack2) point_associate_tobe_mapped(T, p, p);
  std::vector<P> cornerStack, surfStack;
  voxel_grid(cornerStack2, 0.2f, cornerStack);
  voxel_grid(surfStack2, 0.4f, surfStack);
  m.stack += (uint64_t)(cornerStack.size() + surfStack.size());

  if (cornerFromMapNum > 10 && surfFromMapNum > 100) {  // :706-978
    KdTree kdC, kdS;
    kdC.build(cornerFromMap);
    kdS.build(surfFromMap);
    int nI[5];
    float nD[5];
    std::vector<P> cloudOri, coeffSel;
    for (int iterCount = 0; iterCount < cfg.mp_max_iter; ++iterCount) {
      m.iters++;
      cloudOri.clear();
      coeffSel.clear();  // :711-712 rows cleared every iteration (unlike odometry)
      for (const P& pointOri : cornerStack) {  // :714-819
        P pointSel;
        point_associate_to_map(T, pointOri, pointSel);
        int got = kdC.knn(pointSel.x, pointSel.y, pointSel.z, 5, nI, nD);
        if (got < 5 || !(D(nD[4]) < 1.0)) continue;
        float cx = 0, cy = 0, cz = 0;
        for (int j = 0; j < 5; ++j) {
          cx += cornerFromMap[nI[j]].x; cy += cornerFromMap[nI[j]].y; cz += cornerFromMap[nI[j]].z;
        }
        cx /= 5; cy /= 5; cz /= 5;
        float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
        for (int j = 0; j < 5; ++j) {
          float ax = cornerFromMap[nI[j]].x - cx, ay = cornerFromMap[nI[j]].y - cy,
                az = cornerFromMap[nI[j]].z - cz;
          a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
          a22 += ay * ay; a23 += ay * az; a33 += az * az;
        }
        a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
        float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33}, D1[3], V1[9];
        jacobi(A1, 3, D1, V1);
        if (!(D1[0] > 3 * D1[1])) continue;
        float x0 = pointSel.x, y0 = pointSel.y, z0 = pointSel.z;
        float x1 = (float)(D(cx) + 0.1 * D(V1[0])), y1 = (float)(D(cy) + 0.1 * D(V1[1])),
              z1 = (float)(D(cz) + 0.1 * D(V1[2]));
        float x2 = (float)(D(cx) - 0.1 * D(V1[0])), y2 = (float)(D(cy) - 0.1 * D(V1[1])),
              z2 = (float)(D(cz) - 0.1 * D(V1[2]));
        float a012 = (float)std::sqrt(D(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) *
                                            ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                                        ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) *
                                            ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                                        ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) *
                                            ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))));
        float l12 = (float)std::sqrt(D((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) +
                                       (z1 - z2) * (z1 - z2)));
        float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                    (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) /
                   a012 / l12;
        float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                     (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) /
                   a012 / l12;
        float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                     (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) /
                   a012 / l12;
        float ld2 = a012 / l12;
        float sw = (float)(1 - 0.9 * std::fabs(D(ld2)));
        if (D(sw) > 0.1) {
          cloudOri.push_back(pointOri);
          coeffSel.push_back(P{sw * la, sw * lb, sw * lc, sw * ld2});
        }
      }
      for (const P& pointOri : surfStack) {  // :821-877
        P pointSel;
        point_associate_to_map(T, pointOri, pointSel);
        int got = kdS.knn(pointSel.x, pointSel.y, pointSel.z, 5, nI, nD);
        if (got < 5 || !(D(nD[4]) < 1.0)) continue;
        float A0[15], B0[5] = {-1, -1, -1, -1, -1}, X0[3];
        for (int j = 0; j < 5; ++j) {
          A0[j * 3 + 0] = surfFromMap[nI[j]].x;
          A0[j * 3 + 1] = surfFromMap[nI[j]].y;
          A0[j * 3 + 2] = surfFromMap[nI[j]].z;
        }
        qr_solve(A0, B0, 5, 3, X0);
        float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
        float ps = (float)std::sqrt(D(pa * pa + pb * pb + pc * pc));
        pa /= ps; pb /= ps; pc /= ps; pd /= ps;
        bool planeValid = true;
        for (int j = 0; j < 5; ++j) {
          const P& q = surfFromMap[nI[j]];
          if (std::fabs(D(pa * q.x + pb * q.y + pc * q.z + pd)) > 0.2) { planeValid = false; break; }
        }
        if (!planeValid) continue;
        float pd2 = pa * pointSel.x + pb * pointSel.y + pc * pointSel.z + pd;
        float sw = (float)(1 - 0.9 * std::fabs(D(pd2)) /
                                   std::sqrt(std::sqrt(D(pointSel.x * pointSel.x + pointSel.y * pointSel.y +
                                                         pointSel.z * pointSel.z))));
        if (D(sw) > 0.1) {
          cloudOri.push_back(pointOri);
          coeffSel.push_back(P{sw * pa, sw * pb, sw * pc, sw * pd2});
        }
      }
      float srx = (float)dsin(T[0]), crx = (float)dcos(T[0]), sry = (float)dsin(T[1]),
            cry = (float)dcos(T[1]), srz = (float)dsin(T[2]), crz = (float)dcos(T[2]);
      const int selNum = (int)cloudOri.size();
      m.rows_sum += (uint64_t)selNum;
      if (selNum < 50) continue;
      std::vector<float> A((size_t)selNum * 6), Bv(selNum);
      for (int i = 0; i < selNum; ++i) {  // :897-921
        const P& po = cloudOri[i];
        const P& cf = coeffSel[i];
        float arx = (crx * sry * srz * po.x + crx * crz * sry * po.y - srx * sry * po.z) * cf.x +
                    (-srx * srz * po.x - crz * srx * po.y - crx * po.z) * cf.y +
                    (crx * cry * srz * po.x + crx * cry * crz * po.y - cry * srx * po.z) * cf.z;
        float ary = ((cry * srx * srz - crz * sry) * po.x + (sry * srz + cry * crz * srx) * po.y +
                     crx * cry * po.z) * cf.x +
                    ((-cry * crz - srx * sry * srz) * po.x + (cry * srz - crz * srx * sry) * po.y -
                     crx * sry * po.z) * cf.z;
        float arz = ((crz * srx * sry - cry * srz) * po.x + (-cry * crz - srx * sry * srz) * po.y) * cf.x +
                    (crx * crz * po.x - crx * srz * po.y) * cf.y +
                    ((sry * srz + cry * crz * srx) * po.x + (crz * sry - cry * srx * srz) * po.y) * cf.z;
        float* a = &A[(size_t)i * 6];
        a[0] = arx; a[1] = ary; a[2] = arz; a[3] = cf.x; a[4] = cf.y; a[5] = cf.z;
        Bv[i] = -cf.intensity;
      }
      float X[6];
      lm_solve(A, Bv, selNum, iterCount, 100.0f, m.isDegenerate, m.matP, X);
      if (m.isDegenerate) m.deg_steps++;
      for (int q = 0; q < 6; ++q) T[q] += X[q];
      float deltaR = delta_r(X), deltaT = delta_t(X);
      if (D(deltaR) < 0.05 && D(deltaT) < 0.05) break;
    }
    // :199-232 transformUpdate
    if (m.imuLast >= 0) {
      const float scanPeriod = 0.1f;  // const float in laserMapping.cpp:49
      float imuRollLast = 0, imuPitchLast = 0;
      while (m.imuFront != m.imuLast) {
        if (timeLaserOdometry + scanPeriod < m.imuTime[m.imuFront]) break;
        m.imuFront = (m.imuFront + 1) % kImuQue;
      }
      const int F = m.imuFront;
      if (timeLaserOdometry + scanPeriod > m.imuTime[F]) {
        imuRollLast = m.imuRoll[F];
        imuPitchLast = m.imuPitch[F];
      } else {
        const int B = (F + kImuQue - 1) % kImuQue;
        float ratioFront = (float)((timeLaserOdometry + scanPeriod - m.imuTime[B]) / (m.imuTime[F] - m.imuTime[B]));
        float ratioBack = (float)((m.imuTime[F] - timeLaserOdometry - scanPeriod) / (m.imuTime[F] - m.imuTime[B]));
        imuRollLast = m.imuRoll[F] * ratioFront + m.imuRoll[B] * ratioBack;
        imuPitchLast = m.imuPitch[F] * ratioFront + m.imuPitch[B] * ratioBack;
      }
      T[0] = (float)(0.998 * D(T[0]) + 0.002 * D(imuPitchLast));
      T[2] = (float)(0.998 * D(T[2]) + 0.002 * D(imuRollLast));
    }
    for (int i = 0; i < 6; ++i) {
      m.transformBefMapped[i] = m.transformSum[i];
      m.transformAftMapped[i] = T[i];
    }
  }
  // :980-1016 insertion
  for (const P& p : cornerStack) {
    P q;
    point_associate_to_map(T, p, q);
    int ci = cube_of(q.x, m.cenW), cj = cube_of(q.y, m.cenH), ck = cube_of(q.z, m.cenD);
    if (ci >= 0 && ci < kW && cj >= 0 && cj < kH && ck >= 0 && ck < kDp)
      m.corner[ci + kW * cj + kW * kH * ck].push_back(q);
  }
  for (const P& p : surfStack) {
    P q;
    point_associate_to_map(T, p, q);
    int ci = cube_of(q.x, m.cenW), cj = cube_of(q.y, m.cenH), ck = cube_of(q.z, m.cenD);
    if (ci >= 0 && ci < kW && cj >= 0 && cj < kH && ck >= 0 && ck < kDp)
      m.surf[ci + kW * cj + kW * kH * ck].push_back(q);
  }
  // :1018-1036 per valid cube re-downsampling
  std::vector<P> tmp;
  for (int ind : valid) {
    voxel_grid(m.corner[ind], 0.2f, tmp);
    m.corner[ind].swap(tmp);
    voxel_grid(m.surf[ind], 0.4f, tmp);
    m.surf[ind].swap(tmp);
    m.valid_points += (uint64_t)(m.corner[ind].size() + m.surf[ind].size());
  }
  // :1038-1058 /laser_cloud_surround: surround cubes' corner then surf points, VoxelGrid 0.2
  m.mapFrameCount++;
  out.surround_pub = false;
  if (m.mapFrameCount >= 5) {
    m.mapFrameCount = 0;
    std::vector<P> sur2;
    for (int ind : surround) {
      sur2.insert(sur2.end(), m.corner[ind].begin(), m.corner[ind].end());
      sur2.insert(sur2.end(), m.surf[ind].begin(), m.surf[ind].end());
    }
    voxel_grid(sur2, 0.2f, out.surround);
    out.surround_pub = true;
  }
  // :1060-1063
  out.registered.resize(full.size());
  for (size_t i = 0; i < full.size(); ++i) point_associate_to_map(T, full[i], out.registered[i]);
  std::memcpy(out.aft, m.transformAftMapped, sizeof(out.aft));
  std::memcpy(out.bef, m.transformBefMapped, sizeof(out.bef));
}

// nav_msgs pose round trip of the odometry -> mapping / maintenance boundary:
// createQuaternionMsgFromRollPitchYaw(rz, -rx, -ry) + axis permutation (laserOdometry.cpp:858-867)
// then Quaternion(q.z, -q.x, -q.y, q.w).getRPY (laserMapping.cpp:308-318)
void pose_through_msg(const float in[6], float out[6]) {
  Quat g = tf_from_rpy(D(in[2]), -D(in[0]), -D(in[1]));
  Quat msg{-g.y, -g.z, g.x, g.w};
  Quat back{msg.z, -msg.x, -msg.y, msg.w};
  double roll, pitch, yaw;
  tf_get_rpy(back, roll, pitch, yaw);
  out[0] = (float)(-pitch);
  out[1] = (float)(-yaw);
  out[2] = (float)roll;
  out[3] = in[3]; out[4] = in[4]; out[5] = in[5];
}

// ===================================================================== context + C API
struct Oracle {
  Cfg cfg;
  int sr_init_count = 0;
  bool sr_inited = false;
  SrImu imu;
  OdState od;
  MpState mp;
  std::vector<P> surround;  // /laser_cloud_surround of the last mapping frame
  bool surround_pub = false;
  loam_stats stats;
  explicit Oracle(const Cfg& c) : cfg(c) {
    std::memset(&stats, 0, sizeof(stats));
    od.frameCount = c.skip_frame_num;  // int frameCount = skipFrameNum (src/laserOdometry.cpp:407)
  }
};

int write_cloud(const std::vector<P>& v, loam_cloud_out* o) {
  if (o == nullptr) return LOAM_OK;
  if (v.size() > o->capacity) { o->count = (uint32_t)v.size(); return LOAM_E_CAPACITY; }
  if (!v.empty()) std::memcpy(o->pts, v.data(), v.size() * sizeof(P));
  o->count = (uint32_t)v.size();
  return LOAM_OK;
}
std::vector<P> read_cloud(const loam_cloud_out* c) {
  std::vector<P> v;
  if (c && c->count) v.assign((const P*)c->pts, (const P*)c->pts + c->count);
  return v;
}
void to6(const loam_pose6* p, float* f) { std::memcpy(f, p, 6 * sizeof(float)); }
void from6(const float* f, loam_pose6* p) { std::memcpy(p, f, 6 * sizeof(float)); }

}  // namespace

extern "C" {

void oracle_config_default(loam_config* d) {
  std::memset(d, 0, sizeof(*d));
  d->n_rings = 16; d->ring_model = LOAM_RING_VLP16; d->ring_lo_deg = -24.8f; d->ring_hi_deg = 2.0f;
  d->system_delay = 20; d->max_points = 40000; d->od_max_iter = 25; d->mp_max_iter = 10;
  d->skip_frame_num = 1; d->map_capacity = 1u << 21;
}

void* oracle_create(const loam_config* cfg) { return new Oracle(make_cfg(cfg)); }
void oracle_destroy(void* o) { delete static_cast<Oracle*>(o); }

int oracle_scan_registration(void* h, double stamp, loam_cloud_in raw, loam_features* out) {
  Oracle* o = static_cast<Oracle*>(h);
  if (!o->sr_inited) {  // :213-219 (Q1)
    o->sr_init_count++;
    if (o->sr_init_count >= o->cfg.system_delay) o->sr_inited = true;
    return LOAM_E_NOT_READY;
  }
  if (raw.stride_bytes % 4 != 0 || raw.stride_bytes < 12) return LOAM_E_INVAL;
  SrOut r;
  int rc = sr_body(o->cfg, (const float*)raw.data, raw.count, raw.stride_bytes / 4, r, o->imu, stamp);
  if (rc) return rc;
  o->stats.n_raw = raw.count; o->stats.n_ring = r.full.size();
  o->stats.n_sharp = r.sharp.size(); o->stats.n_less_sharp = r.lsharp.size();
  o->stats.n_flat = r.flat.size(); o->stats.n_less_flat = r.lflat.size();
  int e = 0;
  e |= write_cloud(r.full, &out->full);
  e |= write_cloud(r.sharp, &out->sharp);
  e |= write_cloud(r.lsharp, &out->less_sharp);
  e |= write_cloud(r.flat, &out->flat);
  e |= write_cloud(r.lflat, &out->less_flat);
  std::memcpy(out->imu_trans, r.imu_trans, sizeof(out->imu_trans));
  return e ? LOAM_E_CAPACITY : LOAM_OK;
}

int oracle_odometry(void* h, double stamp, const loam_features* in, loam_pose6* sum_out,
                    loam_cloud_out* corner_last, loam_cloud_out* surf_last, loam_cloud_out* full_end,
                    int* published) {
  (void)stamp;
  Oracle* o = static_cast<Oracle*>(h);
  std::vector<P> sharp = read_cloud(&in->sharp), lsharp = read_cloud(&in->less_sharp),
                 flat = read_cloud(&in->flat), lflat = read_cloud(&in->less_flat),
                 full = read_cloud(&in->full);
  OdIn oi{&sharp, &lsharp, &flat, &lflat, &full};
  OdOut oo;
  {  // imuTransHandler (:330-351): the /imu_trans message of this sweep
    const float* t = in->imu_trans;
    OdState& d = o->od;
    d.imuPitchStart = t[0]; d.imuYawStart = t[1]; d.imuRollStart = t[2];
    d.imuPitchLast = t[3]; d.imuYawLast = t[4]; d.imuRollLast = t[5];
    d.imuShiftFromStartX = t[6]; d.imuShiftFromStartY = t[7]; d.imuShiftFromStartZ = t[8];
    d.imuVeloFromStartX = t[9]; d.imuVeloFromStartY = t[10]; d.imuVeloFromStartZ = t[11];
  }
  uint64_t it0 = o->od.iters, as0 = o->od.assoc, rs0 = o->od.rows_sum, q0 = o->od.queries,
           dg0 = o->od.deg_steps, ns0 = o->od.nan_skips;
  o->stats.od_corner_last = o->od.cornerLast.size();
  o->stats.od_surf_last = o->od.surfLast.size();
  od_body(o->cfg, o->od, oi, oo);
  o->stats.od_iters = o->od.iters - it0; o->stats.od_assoc_rounds = o->od.assoc - as0;
  o->stats.od_rows_sum = o->od.rows_sum - rs0; o->stats.od_queries = o->od.queries - q0;
  o->stats.od_degenerate_steps = o->od.deg_steps - dg0; o->stats.od_nan_skips = o->od.nan_skips - ns0;
  {
    const uint64_t as = o->stats.od_assoc_rounds, it = o->stats.od_iters, nq = as ? o->stats.od_queries / as : 0;
    o->stats.od_query_iters = nq * it;
    o->stats.od_row_evals = nq * it * (it + 1) / 2;
  }
  *published = oo.published;
  int e = 0;
  if (oo.published & LOAM_PUB_POSE) from6(oo.sum, sum_out);
  if (oo.published & LOAM_PUB_CLOUDS) {
    e |= write_cloud(oo.cornerLast, corner_last);
    e |= write_cloud(oo.surfLast, surf_last);
  }
  if (oo.published & LOAM_PUB_FULL) e |= write_cloud(oo.full, full_end);
  return e ? LOAM_E_CAPACITY : LOAM_OK;
}

int oracle_mapping(void* h, double stamp, const loam_pose6* odom_sum, const loam_cloud_out* corner_last,
                   const loam_cloud_out* surf_last, const loam_cloud_out* full_end, loam_pose6* aft,
                   loam_pose6* bef, loam_cloud_out* registered) {
  Oracle* o = static_cast<Oracle*>(h);
  float s[6];
  to6(odom_sum, s);
  pose_through_msg(s, o->mp.transformSum);  // laserOdometryHandler :304-321
  std::vector<P> cl = read_cloud(corner_last), sl = read_cloud(surf_last), fl = read_cloud(full_end);
  MpOut mo;
  uint64_t it0 = o->mp.iters, rs0 = o->mp.rows_sum, st0 = o->mp.stack, mp0 = o->mp.map_points,
           vp0 = o->mp.valid_points, dg0 = o->mp.deg_steps, sh0 = o->mp.shifts;
  mp_body(o->cfg, o->mp, cl, sl, fl, mo, stamp);
  o->stats.mp_iters = o->mp.iters - it0; o->stats.mp_rows_sum = o->mp.rows_sum - rs0;
  o->stats.mp_stack = o->mp.stack - st0; o->stats.mp_map_points = o->mp.map_points - mp0;
  o->stats.mp_map_valid_points = o->mp.valid_points - vp0;
  o->stats.mp_degenerate_steps = o->mp.deg_steps - dg0; o->stats.mp_grid_shifts = o->mp.shifts - sh0;
  from6(mo.aft, aft);
  from6(mo.bef, bef);
  o->surround.swap(mo.surround);
  o->surround_pub = mo.surround_pub;
  return write_cloud(mo.registered, registered);
}

// /laser_cloud_surround of the last oracle_mapping frame (src/laserMapping.cpp:1038-1058)
int oracle_mapping_surround(void* h, loam_cloud_out* out, int* published) {
  Oracle* o = static_cast<Oracle*>(h);
  *published = o->surround_pub ? 1 : 0;
  if (!o->surround_pub) {
    out->count = 0;
    return LOAM_OK;
  }
  return write_cloud(o->surround, out);
}

// /imu/data: scanRegistration's imuHandler (:638-660) and laserMapping's (:323-335).
// quat = orientation (x, y, z, w), acc = linear_acceleration (x, y, z), as the sensor_msgs::Imu
// fields (float64)
int oracle_imu(void* h, double stamp, const double* quat, const double* acc) {
  Oracle* o = static_cast<Oracle*>(h);
  sr_imu_handler(o->imu, stamp, quat, acc);
  double roll, pitch, yaw;
  tf_get_rpy(Quat{quat[0], quat[1], quat[2], quat[3]}, roll, pitch, yaw);
  MpState& m = o->mp;
  m.imuLast = (m.imuLast + 1) % kImuQue;
  m.imuTime[m.imuLast] = stamp;
  m.imuRoll[m.imuLast] = (float)roll;
  m.imuPitch[m.imuLast] = (float)pitch;
  return LOAM_OK;
}

int oracle_maintenance(const loam_pose6* odom_sum, const loam_pose6* bef, const loam_pose6* aft,
                       loam_pose6* integrated) {
  // transformMaintenance.cpp:147-203: Sum and Aft arrive through the quaternion messages, Bef
  // through the twist fields (exact)
  MpState m;  // reuse transformAssociateToMap (identical algebra, :60-145)
  float s[6], a[6];
  to6(odom_sum, s);
  to6(aft, a);
  pose_through_msg(s, m.transformSum);
  pose_through_msg(a, m.transformAftMapped);
  to6(bef, m.transformBefMapped);
  transform_associate_to_map(m);
  from6(m.transformTobeMapped, integrated);
  return LOAM_OK;
}

int oracle_get_stats(void* h, loam_stats* st) {
  *st = static_cast<Oracle*>(h)->stats;
  return LOAM_OK;
}

// One config-4 problem: SR(prev), SR(cur); odometry seeded from prev as a solved
// zero-increment frame, then one loop body on cur; mapping of prev into an empty map, then one
// mapping body for cur.  Outputs the odometry transformSum and the mapped (Aft) pose.
int oracle_problem(const loam_config* cfg, loam_cloud_in prev, loam_cloud_in cur, loam_pose6* od_sum,
                   loam_pose6* aft, loam_stats* st) {
  Cfg c = make_cfg(cfg);
  SrOut a, b;
  SrImu no_imu;  // config 4 has no IMU
  int rc = sr_body(c, (const float*)prev.data, prev.count, prev.stride_bytes / 4, a, no_imu, 0.0);
  if (rc) return rc;
  rc = sr_body(c, (const float*)cur.data, cur.count, cur.stride_bytes / 4, b, no_imu, 0.1);
  if (rc) return rc;
  OdState od;
  od.inited = true;
  od.cornerLast.resize(a.lsharp.size());
  od.surfLast.resize(a.lflat.size());
  for (size_t i = 0; i < a.lsharp.size(); ++i) transform_to_end(od, a.lsharp[i], od.cornerLast[i]);
  for (size_t i = 0; i < a.lflat.size(); ++i) transform_to_end(od, a.lflat[i], od.surfLast[i]);
  std::vector<P> prevFull(a.full.size());
  for (size_t i = 0; i < a.full.size(); ++i) transform_to_end(od, a.full[i], prevFull[i]);
  od.cornerLastNum = (int)od.cornerLast.size();
  od.surfLastNum = (int)od.surfLast.size();
  if (od.cornerLastNum > 10 && od.surfLastNum > 100) {
    od.kdCorner.build(od.cornerLast);
    od.kdSurf.build(od.surfLast);
  }
  od.frameCount = c.skip_frame_num;  // the cur frame publishes its clouds
  OdIn oi{&b.sharp, &b.lsharp, &b.flat, &b.lflat, &b.full};
  OdOut oo;
  MpState mp;
  MpOut m0, m1;
  const std::vector<P> prevCorner = od.cornerLast, prevSurf = od.surfLast;
  od_body(c, od, oi, oo);
  // mapping: prev frame at the origin (empty map: no L-M), then cur with the odometry pose
  float zero[6] = {0, 0, 0, 0, 0, 0};
  pose_through_msg(zero, mp.transformSum);
  mp_body(c, mp, prevCorner, prevSurf, prevFull, m0);
  pose_through_msg(oo.sum, mp.transformSum);
  mp_body(c, mp, oo.cornerLast, oo.surfLast, oo.full, m1);
  from6(oo.sum, od_sum);
  from6(m1.aft, aft);
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->n_raw = prev.count + cur.count;
    st->n_ring = a.full.size() + b.full.size();
    st->n_sharp = a.sharp.size() + b.sharp.size();
    st->n_less_sharp = a.lsharp.size() + b.lsharp.size();
    st->n_flat = a.flat.size() + b.flat.size();
    st->n_less_flat = a.lflat.size() + b.lflat.size();
    st->od_iters = od.iters; st->od_assoc_rounds = od.assoc; st->od_rows_sum = od.rows_sum;
    st->od_corner_last = prevCorner.size(); st->od_surf_last = prevSurf.size();
    st->od_queries = od.queries;
    {
      const uint64_t nq = od.assoc ? (uint64_t)od.queries / od.assoc : 0, it = od.iters;
      st->od_query_iters = nq * it;
      st->od_row_evals = nq * it * (it + 1) / 2;
    }
    st->mp_iters = mp.iters; st->mp_rows_sum = mp.rows_sum; st->mp_stack = mp.stack;
    st->mp_map_points = mp.map_points; st->mp_map_valid_points = mp.valid_points;
    st->od_degenerate_steps = od.deg_steps; st->od_nan_skips = od.nan_skips;
    st->mp_degenerate_steps = mp.deg_steps; st->mp_grid_shifts = mp.shifts;
  }
  return LOAM_OK;
}

// oracle_problem with the odometry's L-M solution (transform[6]) replaced by od_transform before it
// is accumulated and used for TransformToEnd: the reference's mapping for another odometry result
// (tests/test_gpu_moments.py replays the engine's per-query-moments odometry through it)
int oracle_problem_with_od(const loam_config* cfg, loam_cloud_in prev, loam_cloud_in cur,
                           const loam_pose6* od_transform, loam_pose6* od_sum, loam_pose6* aft, loam_stats* st) {
  g_od_override = &od_transform->rx;
  const int rc = oracle_problem(cfg, prev, cur, od_sum, aft, st);
  g_od_override = nullptr;
  return rc;
}

// ---- component hooks for the oracle's own known-answer tests
int oracle_voxel_grid(const float* in, int n, float leaf, float* out, int cap) {
  std::vector<P> v((const P*)in, (const P*)in + n), o;
  voxel_grid(v, leaf, o);
  if ((int)o.size() > cap) return -(int)o.size();
  std::memcpy(out, o.data(), o.size() * sizeof(P));
  return (int)o.size();
}
int oracle_knn(const float* pts, int n, const float* q, int nq, int k, int* idx, float* d) {
  std::vector<P> v((const P*)pts, (const P*)pts + n);
  KdTree t;
  t.build(v);
  for (int i = 0; i < nq; ++i) {
    int got = t.knn(q[4 * i], q[4 * i + 1], q[4 * i + 2], k, idx + i * k, d + i * k);
    for (int j = got; j < k; ++j) { idx[i * k + j] = -1; d[i * k + j] = INFINITY; }
  }
  return 0;
}
int oracle_qr_solve(const float* A, const float* b, int m, int n, float* x) {
  return qr_solve(A, b, m, n, x) ? 1 : 0;
}
void oracle_jacobi(const float* A, int n, float* W, float* V) { jacobi(A, n, W, V); }
int oracle_lu_inv(const float* A, int n, float* inv) { return lu_inv(A, n, inv) ? 1 : 0; }
void oracle_pose_through_msg(const float* in, float* out) { pose_through_msg(in, out); }
// the published orientation of a pose message (laserOdometry.cpp:858-864): (-q.y, -q.z, q.x, q.w)
// of createQuaternionMsgFromRollPitchYaw(rz, -rx, -ry)
void oracle_msg_orientation(const float* in, double* xyzw) {
  Quat g = tf_from_rpy(D(in[2]), -D(in[0]), -D(in[1]));
  xyzw[0] = -g.y; xyzw[1] = -g.z; xyzw[2] = g.x; xyzw[3] = g.w;
}

}  // extern "C"
