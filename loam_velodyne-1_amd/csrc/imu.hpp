// IMU de-skew of scanRegistration (src/scanRegistration.cpp:68-209, :286-349, :614-660) and the
// IMU queue of laserMapping (src/laserMapping.cpp:101-108, :199-232, :323-335).
//
// The queues are fed on the host (loam_imu, one message at a time: AccumulateIMUShift depends on
// the previous entry).  Scan registration runs the per-point part on the device: the reference's
// forward-only imuPointerFront walk is a running maximum of "first queue entry later than this
// point" over the points in input order, so every point finds its entry by binary search and a
// block-wide max-scan restores the walk.  Float sin / cos are the glibc-identical restatements
// (dev_common.hpp) because scanRegistration binds std::sin / std::cos to floats.
#ifndef LOAM_IMU_HPP
#define LOAM_IMU_HPP

#include "dev_common.hpp"

namespace loamimu {

using loamdev::D;
using loamdev::cosf_glibc;
using loamdev::sinf_glibc;

constexpr int kQue = 200;  // imuQueLength (:70)

// scanRegistration's IMU globals (:68-97); uploaded to the device per sweep, read back after
struct SrQueue {
  double time[kQue];
  float roll[kQue], pitch[kQue], yaw[kQue];
  float accX[kQue], accY[kQue], accZ[kQue];
  float veloX[kQue], veloY[kQue], veloZ[kQue];
  float shiftX[kQue], shiftY[kQue], shiftZ[kQue];
  int front, last;
  // Start (:72-78), Cur of the last processed point (:73-82), ShiftFromStart / VeloFromStart (:83-84)
  float rollStart, pitchStart, yawStart, veloXStart, veloYStart, veloZStart, shiftXStart, shiftYStart,
      shiftZStart;
  float rollCur, pitchCur, yawCur, veloXCur, veloYCur, veloZCur, shiftXCur, shiftYCur, shiftZCur;
  float shiftFSX, shiftFSY, shiftFSZ, veloFSX, veloFSY, veloFSZ;
};

// laserMapping's queue (:101-108)
struct MpQueue {
  double time[kQue];
  float roll[kQue], pitch[kQue];
  int front, last;
};

// one point's interpolated IMU state (the *Cur globals)
struct Cur {
  float roll, pitch, yaw, vx, vy, vz, sx, sy, sz;
};

// :162-200 AccumulateIMUShift (host)
inline void accumulate_shift(SrQueue& m) {
  const int L = m.last;
  float roll = m.roll[L], pitch = m.pitch[L], yaw = m.yaw[L];
  float accX = m.accX[L], accY = m.accY[L], accZ = m.accZ[L];
  float x1 = cosf_glibc(roll) * accX - sinf_glibc(roll) * accY;
  float y1 = sinf_glibc(roll) * accX + cosf_glibc(roll) * accY;
  float z1 = accZ;
  float x2 = x1;
  float y2 = cosf_glibc(pitch) * y1 - sinf_glibc(pitch) * z1;
  float z2 = sinf_glibc(pitch) * y1 + cosf_glibc(pitch) * z1;
  accX = cosf_glibc(yaw) * x2 + sinf_glibc(yaw) * z2;
  accY = y2;
  accZ = -sinf_glibc(yaw) * x2 + cosf_glibc(yaw) * z2;
  const int B = (L + kQue - 1) % kQue;
  const double timeDiff = m.time[L] - m.time[B];
  if (timeDiff < 0.1) {  // scanPeriod (double, :55)
    m.shiftX[L] = (float)(D(m.shiftX[B]) + D(m.veloX[B]) * timeDiff + D(accX) * timeDiff * timeDiff / 2);
    m.shiftY[L] = (float)(D(m.shiftY[B]) + D(m.veloY[B]) * timeDiff + D(accY) * timeDiff * timeDiff / 2);
    m.shiftZ[L] = (float)(D(m.shiftZ[B]) + D(m.veloZ[B]) * timeDiff + D(accZ) * timeDiff * timeDiff / 2);
    m.veloX[L] = (float)(D(m.veloX[B]) + D(accX) * timeDiff);
    m.veloY[L] = (float)(D(m.veloY[B]) + D(accY) * timeDiff);
    m.veloZ[L] = (float)(D(m.veloZ[B]) + D(accZ) * timeDiff);
  }
}

// :638-660 imuHandler (host); roll / pitch / yaw from the message quaternion by tf getRPY
inline void sr_push(SrQueue& m, double stamp, double roll, double pitch, double yaw, const double* acc) {
  const float accX = (float)(acc[1] - sin(roll) * cos(pitch) * 9.81);
  const float accY = (float)(acc[2] - cos(roll) * cos(pitch) * 9.81);
  const float accZ = (float)(acc[0] + sin(pitch) * 9.81);
  m.last = (m.last + 1) % kQue;
  m.time[m.last] = stamp;
  m.roll[m.last] = (float)roll;
  m.pitch[m.last] = (float)pitch;
  m.yaw[m.last] = (float)yaw;
  m.accX[m.last] = accX;
  m.accY[m.last] = accY;
  m.accZ[m.last] = accZ;
  accumulate_shift(m);
}

// :323-335 (host)
inline void mp_push(MpQueue& m, double stamp, double roll, double pitch) {
  m.last = (m.last + 1) % kQue;
  m.time[m.last] = stamp;
  m.roll[m.last] = (float)roll;
  m.pitch[m.last] = (float)pitch;
}

// :199-226 (host): the IMU roll / pitch at timeLaserOdometry + scanPeriod and the advanced front
// pointer; the caller commits the pointer only when transformUpdate runs
inline bool mp_lookup(const MpQueue& m, double timeLaserOdometry, float& rollLast, float& pitchLast, int& front) {
  if (m.last < 0) return false;
  const float scanPeriod = 0.1f;  // const float in laserMapping.cpp:49
  front = m.front;
  while (front != m.last) {
    if (timeLaserOdometry + scanPeriod < m.time[front]) break;
    front = (front + 1) % kQue;
  }
  if (timeLaserOdometry + scanPeriod > m.time[front]) {
    rollLast = m.roll[front];
    pitchLast = m.pitch[front];
  } else {
    const int B = (front + kQue - 1) % kQue;
    const float ratioFront = (float)((timeLaserOdometry + scanPeriod - m.time[B]) / (m.time[front] - m.time[B]));
    const float ratioBack = (float)((m.time[front] - timeLaserOdometry - scanPeriod) / (m.time[front] - m.time[B]));
    rollLast = m.roll[front] * ratioFront + m.roll[B] * ratioBack;
    pitchLast = m.pitch[front] * ratioFront + m.pitch[B] * ratioBack;
  }
  return true;
}

// first logical queue position k in [0, L] (from `front0`) whose stamp is later than t, else L: the
// stop of the :288-293 walk started at front0 (stamps non-decreasing, loam_imu enforces it)
LOAM_HD int first_later(const SrQueue& m, int front0, double t) {
  const int L = (m.last - front0 + kQue) % kQue;
  int lo = 0, hi = L;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (t < m.time[(front0 + mid) % kQue]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// :295-331 the point's interpolated state from queue entry F
LOAM_HD Cur interpolate(const SrQueue& m, int F, double timeScanCur, float pointTime) {
  Cur c;
  const double tp = timeScanCur + pointTime;
  if (tp > m.time[F]) {
    c.roll = m.roll[F]; c.pitch = m.pitch[F]; c.yaw = m.yaw[F];
    c.vx = m.veloX[F]; c.vy = m.veloY[F]; c.vz = m.veloZ[F];
    c.sx = m.shiftX[F]; c.sy = m.shiftY[F]; c.sz = m.shiftZ[F];
    return c;
  }
  const int B = (F + kQue - 1) % kQue;
  const float ratioFront = (float)((tp - m.time[B]) / (m.time[F] - m.time[B]));
  const float ratioBack = (float)((m.time[F] - timeScanCur - pointTime) / (m.time[F] - m.time[B]));
  c.roll = m.roll[F] * ratioFront + m.roll[B] * ratioBack;
  c.pitch = m.pitch[F] * ratioFront + m.pitch[B] * ratioBack;
  if (D(m.yaw[F] - m.yaw[B]) > M_PI)
    c.yaw = (float)(D(m.yaw[F] * ratioFront) + (D(m.yaw[B]) + 2 * M_PI) * D(ratioBack));
  else if (D(m.yaw[F] - m.yaw[B]) < -M_PI)
    c.yaw = (float)(D(m.yaw[F] * ratioFront) + (D(m.yaw[B]) - 2 * M_PI) * D(ratioBack));
  else
    c.yaw = m.yaw[F] * ratioFront + m.yaw[B] * ratioBack;
  c.vx = m.veloX[F] * ratioFront + m.veloX[B] * ratioBack;
  c.vy = m.veloY[F] * ratioFront + m.veloY[B] * ratioBack;
  c.vz = m.veloZ[F] * ratioFront + m.veloZ[B] * ratioBack;
  c.sx = m.shiftX[F] * ratioFront + m.shiftX[B] * ratioBack;
  c.sy = m.shiftY[F] * ratioFront + m.shiftY[B] * ratioBack;
  c.sz = m.shiftZ[F] * ratioFront + m.shiftZ[B] * ratioBack;
  return c;
}

// the Start values and their sines / cosines (per sweep)
struct Start {
  float roll, pitch, yaw, vx, vy, vz, sx, sy, sz;
  float cr, sr, cp, sp, cy, sy_;
};
LOAM_HD Start make_start(const Cur& c) {
  Start s;
  s.roll = c.roll; s.pitch = c.pitch; s.yaw = c.yaw;
  s.vx = c.vx; s.vy = c.vy; s.vz = c.vz;
  s.sx = c.sx; s.sy = c.sy; s.sz = c.sz;
  s.cr = cosf_glibc(s.roll); s.sr = sinf_glibc(s.roll);
  s.cp = cosf_glibc(s.pitch); s.sp = sinf_glibc(s.pitch);
  s.cy = cosf_glibc(s.yaw); s.sy_ = sinf_glibc(s.yaw);
  return s;
}

// :111-127 ShiftToStartIMU and :129-145 VeloToStartIMU: fs = (shift xyz, velo xyz) from start
LOAM_HD void to_start(const Start& S, const Cur& c, float pointTime, float* fs) {
  float ex = c.sx - S.sx - S.vx * pointTime;
  float ey = c.sy - S.sy - S.vy * pointTime;
  float ez = c.sz - S.sz - S.vz * pointTime;
  for (int k = 0; k < 2; ++k) {
    if (k == 1) { ex = c.vx - S.vx; ey = c.vy - S.vy; ez = c.vz - S.vz; }
    float x1 = S.cy * ex - S.sy_ * ez;
    float y1 = ey;
    float z1 = S.sy_ * ex + S.cy * ez;
    float x2 = x1;
    float y2 = S.cp * y1 + S.sp * z1;
    float z2 = -S.sp * y1 + S.cp * z1;
    fs[3 * k + 0] = S.cr * x2 + S.sr * y2;
    fs[3 * k + 1] = -S.sr * x2 + S.cr * y2;
    fs[3 * k + 2] = z2;
  }
}

// :147-160 TransformToStartIMU
LOAM_HD float4 transform_to_start(const Start& S, const Cur& c, const float* fs, float4 p) {
  const float cr = cosf_glibc(c.roll), sr = sinf_glibc(c.roll);
  const float cp = cosf_glibc(c.pitch), sp = sinf_glibc(c.pitch);
  const float cy = cosf_glibc(c.yaw), sy = sinf_glibc(c.yaw);
  float x1 = cr * p.x - sr * p.y;
  float y1 = sr * p.x + cr * p.y;
  float z1 = p.z;
  float x2 = x1;
  float y2 = cp * y1 - sp * z1;
  float z2 = sp * y1 + cp * z1;
  float x3 = cy * x2 + sy * z2;
  float y3 = y2;
  float z3 = -sy * x2 + cy * z2;
  float x4 = S.cy * x3 - S.sy_ * z3;
  float y4 = y3;
  float z4 = S.sy_ * x3 + S.cy * z3;
  float x5 = x4;
  float y5 = S.cp * y4 + S.sp * z4;
  float z5 = -S.sp * y4 + S.cp * z4;
  float4 o;
  o.x = S.cr * x5 + S.sr * y5 + fs[0];
  o.y = -S.sr * x5 + S.cr * y5 + fs[1];
  o.z = z5 + fs[2];
  o.w = p.w;
  return o;
}

}  // namespace loamimu

#endif
