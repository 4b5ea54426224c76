// Scalar pose algebra of the reference, callable from kernels and from host code.
// Float variables with the reference toolchain's double-evaluated libm calls (see dev_common.hpp).
//   TransformToStart / TransformToEnd      src/laserOdometry.cpp:101-194
//   PluginIMURotation / AccumulateRotation src/laserOdometry.cpp:196-273
//   pose accumulation                      src/laserOdometry.cpp:830-856
//   transformAssociateToMap                src/laserMapping.cpp:110-197 (= transformMaintenance.cpp:60-145)
//   pointAssociateToMap / ...TobeMapped    src/laserMapping.cpp:234-272
//   nav_msgs quaternion round trip         src/laserOdometry.cpp:858-867 -> src/laserMapping.cpp:308-318
#ifndef LOAM_POSE_MATH_HPP
#define LOAM_POSE_MATH_HPP

#if defined(LOAM_DIAG_END_NOTRIG) && !defined(LOAM_EXPERIMENT_BUILD)
#error "LOAM_DIAG_END_NOTRIG is a timing diagnostic (wrong results): tools/build_variant.sh only"
#endif

#include "dev_common.hpp"

namespace loampose {

using loamdev::D;
using loamdev::dcos;
using loamdev::dsin;
using loamdev::dsincos;

// /imu_trans values (zero without IMU); layout of loam_features.imu_trans
struct Imu {
  float pitchStart, yawStart, rollStart, pitchLast, yawLast, rollLast;
  float shiftX, shiftY, shiftZ, veloX, veloY, veloZ;
};

LOAM_HD float4 transform_to_start(const float* t, float4 pi) {
  float s = 10 * (pi.w - (int)pi.w);
  float rx = s * t[0], ry = s * t[1], rz = s * t[2];
  float tx = s * t[3], ty = s * t[4], tz = s * t[5];
  double sx, cx, sy, cy, sz, cz;
  dsincos(rx, sx, cx);
  dsincos(ry, sy, cy);
  dsincos(rz, sz, cz);
  float x1 = (float)(cz * D(pi.x - tx) + sz * D(pi.y - ty));
  float y1 = (float)(-sz * D(pi.x - tx) + cz * D(pi.y - ty));
  float z1 = (pi.z - tz);
  float y2 = (float)(cx * D(y1) + sx * D(z1));
  float z2 = (float)(-sx * D(y1) + cx * D(z1));
  float4 o;
  o.x = (float)(cy * D(x1) - sy * D(z2));
  o.y = y2;
  o.z = (float)(sy * D(x1) + cy * D(z2));
  o.w = pi.w;
  return o;
}

// the trigonometry of TransformToEnd that does not depend on the point: the transform's own
// angles (second rotation) and the six IMU angles, evaluated once per thread
struct EndRot {
  double crx, srx, cry, sry, crz, srz;
  double crs, srs, cps, sps, cys, sys, cyl, syl, cpl, spl, crl, srl;  // roll/pitch/yaw Start, yaw/pitch/roll Last
};
LOAM_HD EndRot end_rot(const float* t, const Imu& m) {
  EndRot e;
  dsincos(t[0], e.srx, e.crx);
  dsincos(t[1], e.sry, e.cry);
  dsincos(t[2], e.srz, e.crz);
  dsincos(m.rollStart, e.srs, e.crs);
  dsincos(m.pitchStart, e.sps, e.cps);
  dsincos(m.yawStart, e.sys, e.cys);
  dsincos(m.yawLast, e.syl, e.cyl);
  dsincos(m.pitchLast, e.spl, e.cpl);
  dsincos(m.rollLast, e.srl, e.crl);
  return e;
}

// end_rot by a converged wave: lane k < 9 evaluates the k-th of its nine sines / cosines (the same
// calls, so the same values) and every lane takes them by readlane — one library sincos per wave
// instead of nine per lane (k_mp_register / k_od_end run it once per workgroup)
LOAM_D EndRot end_rot_wave(const float* t, const Imu& m) {
  const int lane = __lane_id();
  const float a = lane == 0 ? t[0] : lane == 1 ? t[1] : lane == 2 ? t[2] : lane == 3 ? m.rollStart :
                  lane == 4 ? m.pitchStart : lane == 5 ? m.yawStart : lane == 6 ? m.yawLast :
                  lane == 7 ? m.pitchLast : m.rollLast;
  double sv, cv;
  dsincos(a, sv, cv);
  auto rl = [&](double v, int k) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, k), hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
  };
  EndRot e;
  e.srx = rl(sv, 0); e.crx = rl(cv, 0);
  e.sry = rl(sv, 1); e.cry = rl(cv, 1);
  e.srz = rl(sv, 2); e.crz = rl(cv, 2);
  e.srs = rl(sv, 3); e.crs = rl(cv, 3);
  e.sps = rl(sv, 4); e.cps = rl(cv, 4);
  e.sys = rl(sv, 5); e.cys = rl(cv, 5);
  e.syl = rl(sv, 6); e.cyl = rl(cv, 6);
  e.spl = rl(sv, 7); e.cpl = rl(cv, 7);
  e.srl = rl(sv, 8); e.crl = rl(cv, 8);
  return e;
}

// TransformToEnd (:126-194).  `zero`: the transform is known to be all +0, so for s >= 0 the
// scaled angles are +0 and their sines / cosines exactly 0 / 1 (no library calls).
LOAM_HD float4 transform_to_end(const float* t, const Imu& m, const EndRot& e, float4 pi, bool zero) {
  float s = 10 * (pi.w - (int)pi.w);
  float rx = s * t[0], ry = s * t[1], rz = s * t[2];
  float tx = s * t[3], ty = s * t[4], tz = s * t[5];
  double cx, sx, cy, sy, cz, sz;
  if (zero && s >= 0) {
    cx = cy = cz = 1.0;
    sx = sy = sz = 0.0;
#ifdef LOAM_DIAG_END_NOTRIG
  } else if (true) {  // timing diagnostic only (wrong results): the per-point trigonometry left out
    sx = rx; sy = ry; sz = rz;
    cx = cy = cz = 1.0;
#endif
  } else {
    dsincos(rx, sx, cx);
    dsincos(ry, sy, cy);
    dsincos(rz, sz, cz);
  }
  float x1 = (float)(cz * D(pi.x - tx) + sz * D(pi.y - ty));
  float y1 = (float)(-sz * D(pi.x - tx) + cz * D(pi.y - ty));
  float z1 = (pi.z - tz);
  float y2 = (float)(cx * D(y1) + sx * D(z1));
  float z2 = (float)(-sx * D(y1) + cx * D(z1));
  float x3 = (float)(cy * D(x1) - sy * D(z2));
  float y3 = y2;
  float z3 = (float)(sy * D(x1) + cy * D(z2));
  tx = t[3]; ty = t[4]; tz = t[5];
  float x4 = (float)(e.cry * D(x3) + e.sry * D(z3));
  float z4 = (float)(-e.sry * D(x3) + e.cry * D(z3));
  float y5 = (float)(e.crx * D(y3) - e.srx * D(z4));
  float z5 = (float)(e.srx * D(y3) + e.crx * D(z4));
  float x6 = (float)(e.crz * D(x4) - e.srz * D(y5) + D(tx));
  float y6 = (float)(e.srz * D(x4) + e.crz * D(y5) + D(ty));
  float z6 = z5 + tz;
  float x7 = (float)(e.crs * D(x6 - m.shiftX) - e.srs * D(y6 - m.shiftY));
  float y7 = (float)(e.srs * D(x6 - m.shiftX) + e.crs * D(y6 - m.shiftY));
  float z7 = z6 - m.shiftZ;
  float y8 = (float)(e.cps * D(y7) - e.sps * D(z7));
  float z8 = (float)(e.sps * D(y7) + e.cps * D(z7));
  float x9 = (float)(e.cys * D(x7) + e.sys * D(z8));
  float z9 = (float)(-e.sys * D(x7) + e.cys * D(z8));
  float x10 = (float)(e.cyl * D(x9) - e.syl * D(z9));
  float z10 = (float)(e.syl * D(x9) + e.cyl * D(z9));
  float y11 = (float)(e.cpl * D(y8) + e.spl * D(z10));
  float z11 = (float)(-e.spl * D(y8) + e.cpl * D(z10));
  float4 o;
  o.x = (float)(e.crl * D(x10) + e.srl * D(y11));
  o.y = (float)(-e.srl * D(x10) + e.crl * D(y11));
  o.z = z11;
  o.w = (float)(int)pi.w;
  return o;
}

LOAM_HD float4 transform_to_end(const float* t, const Imu& m, float4 pi) {
  return transform_to_end(t, m, end_rot(t, m), pi, false);
}

LOAM_HD void plugin_imu_rotation(float bcx, float bcy, float bcz, float blx, float bly, float blz,
                                 float alx, float aly, float alz, float& acx, float& acy,
                                 float& acz) {
  float sbcx = (float)dsin(bcx), cbcx = (float)dcos(bcx), sbcy = (float)dsin(bcy),
        cbcy = (float)dcos(bcy), sbcz = (float)dsin(bcz), cbcz = (float)dcos(bcz);
  float sblx = (float)dsin(blx), cblx = (float)dcos(blx), sbly = (float)dsin(bly),
        cbly = (float)dcos(bly), sblz = (float)dsin(blz), cblz = (float)dcos(blz);
  float salx = (float)dsin(alx), calx = (float)dcos(alx), saly = (float)dsin(aly),
        caly = (float)dcos(aly), salz = (float)dsin(alz), calz = (float)dcos(alz);
  // shared sub-terms, in the reference's evaluation order
  float u1 = salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly;
  float u2 = calx * saly * (cbly * sblz - cblz * sblx * sbly) -
             calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx;
  float u3 = calx * caly * (cblz * sbly - cbly * sblx * sblz) -
             calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz;
  float srx = -sbcx * u1 - cbcx * cbcz * u2 - cbcx * sbcz * u3;
  acx = (float)(-asin(D(srx)));
  float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * u2 - (cbcy * cbcz + sbcx * sbcy * sbcz) * u3 +
                 cbcx * sbcy * u1;
  float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * u3 - (sbcy * sbcz + cbcy * cbcz * sbcx) * u2 +
                 cbcx * cbcy * u1;
  acy = (float)atan2(D(srycrx) / dcos(acx), D(crycrx) / dcos(acx));
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
  acz = (float)atan2(D(srzcrx) / dcos(acx), D(crzcrx) / dcos(acx));
}

LOAM_HD void accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz,
                                 float& ox, float& oy, float& oz) {
  const double scx = dsin(cx), ccx = dcos(cx), scy = dsin(cy), ccy = dcos(cy), scz = dsin(cz),
               ccz = dcos(cz);
  const double slx = dsin(lx), clx = dcos(lx), sly = dsin(ly), cly = dcos(ly), slz = dsin(lz),
               clz = dcos(lz);
  float srx = (float)(clx * ccx * sly * scz - ccx * ccz * slx - clx * cly * scx);
  ox = (float)(-asin(D(srx)));
  float srycrx = (float)(slx * (ccy * scz - ccz * scx * scy) + clx * sly * (ccy * ccz + scx * scy * scz) +
                         clx * cly * ccx * scy);
  float crycrx = (float)(clx * cly * ccx * ccy - clx * sly * (ccz * scy - ccy * scx * scz) -
                         slx * (scy * scz + ccy * ccz * scx));
  oy = (float)atan2(D(srycrx) / dcos(ox), D(crycrx) / dcos(ox));
  float srzcrx = (float)(scx * (clz * sly - cly * slx * slz) + ccx * scz * (cly * clz + slx * sly * slz) +
                         clx * ccx * ccz * slz);
  float crzcrx = (float)(clx * clz * ccx * ccz - ccx * scz * (cly * slz - clz * slx * sly) -
                         scx * (sly * slz + cly * clz * slx));
  oz = (float)atan2(D(srzcrx) / dcos(ox), D(crzcrx) / dcos(ox));
}

// pose accumulation of one odometry frame into transformSum (:830-856)
LOAM_HD void accumulate_pose(const float* transform, const Imu& m, float* sum) {
  float rx, ry, rz;
  accumulate_rotation(sum[0], sum[1], sum[2], -transform[0], (float)(-D(transform[1]) * 1.05),
                      -transform[2], rx, ry, rz);
  float x1 = (float)(dcos(rz) * D(transform[3] - m.shiftX) - dsin(rz) * D(transform[4] - m.shiftY));
  float y1 = (float)(dsin(rz) * D(transform[3] - m.shiftX) + dcos(rz) * D(transform[4] - m.shiftY));
  float z1 = (float)(D(transform[5]) * 1.05 - D(m.shiftZ));
  float y2 = (float)(dcos(rx) * D(y1) - dsin(rx) * D(z1));
  float z2 = (float)(dsin(rx) * D(y1) + dcos(rx) * D(z1));
  float tx = (float)(D(sum[3]) - (dcos(ry) * D(x1) + dsin(ry) * D(z2)));
  float ty = sum[4] - y2;
  float tz = (float)(D(sum[5]) - (-dsin(ry) * D(x1) + dcos(ry) * D(z2)));
  plugin_imu_rotation(rx, ry, rz, m.pitchStart, m.yawStart, m.rollStart, m.pitchLast, m.yawLast,
                      m.rollLast, rx, ry, rz);
  sum[0] = rx; sum[1] = ry; sum[2] = rz;
  sum[3] = tx; sum[4] = ty; sum[5] = tz;
}

// transformAssociateToMap: T (TobeMapped or Mapped) from Sum, Bef, Aft; incre = transformIncre
LOAM_HD void associate_to_map(const float* S, const float* B, const float* A, float* incre, float* T) {
  float x1 = (float)(dcos(S[1]) * D(B[3] - S[3]) - dsin(S[1]) * D(B[5] - S[5]));
  float y1 = B[4] - S[4];
  float z1 = (float)(dsin(S[1]) * D(B[3] - S[3]) + dcos(S[1]) * D(B[5] - S[5]));
  float y2 = (float)(dcos(S[0]) * D(y1) + dsin(S[0]) * D(z1));
  float z2 = (float)(-dsin(S[0]) * D(y1) + dcos(S[0]) * D(z1));
  incre[3] = (float)(dcos(S[2]) * D(x1) + dsin(S[2]) * D(y2));
  incre[4] = (float)(-dsin(S[2]) * D(x1) + dcos(S[2]) * D(y2));
  incre[5] = z2;
  float sbcx = (float)dsin(S[0]), cbcx = (float)dcos(S[0]), sbcy = (float)dsin(S[1]),
        cbcy = (float)dcos(S[1]), sbcz = (float)dsin(S[2]), cbcz = (float)dcos(S[2]);
  float sblx = (float)dsin(B[0]), cblx = (float)dcos(B[0]), sbly = (float)dsin(B[1]),
        cbly = (float)dcos(B[1]), sblz = (float)dsin(B[2]), cblz = (float)dcos(B[2]);
  float salx = (float)dsin(A[0]), calx = (float)dcos(A[0]), saly = (float)dsin(A[1]),
        caly = (float)dcos(A[1]), salz = (float)dsin(A[2]), calz = (float)dcos(A[2]);
  float u1 = salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly;
  float u2 = calx * saly * (cbly * sblz - cblz * sblx * sbly) -
             calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx;
  float u3 = calx * caly * (cblz * sbly - cbly * sblx * sblz) -
             calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz;
  float srx = -sbcx * u1 - cbcx * cbcz * u2 - cbcx * sbcz * u3;
  T[0] = (float)(-asin(D(srx)));
  float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * u2 - (cbcy * cbcz + sbcx * sbcy * sbcz) * u3 +
                 cbcx * sbcy * u1;
  float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * u3 - (sbcy * sbcz + cbcy * cbcz * sbcx) * u2 +
                 cbcx * cbcy * u1;
  T[1] = (float)atan2(D(srycrx) / dcos(T[0]), D(crycrx) / dcos(T[0]));
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
  T[2] = (float)atan2(D(srzcrx) / dcos(T[0]), D(crzcrx) / dcos(T[0]));
  x1 = (float)(dcos(T[2]) * D(incre[3]) - dsin(T[2]) * D(incre[4]));
  y1 = (float)(dsin(T[2]) * D(incre[3]) + dcos(T[2]) * D(incre[4]));
  z1 = incre[5];
  y2 = (float)(dcos(T[0]) * D(y1) - dsin(T[0]) * D(z1));
  z2 = (float)(dsin(T[0]) * D(y1) + dcos(T[0]) * D(z1));
  T[3] = (float)(D(A[3]) - (dcos(T[1]) * D(x1) + dsin(T[1]) * D(z2)));
  T[4] = A[4] - y2;
  T[5] = (float)(D(A[5]) - (-dsin(T[1]) * D(x1) + dcos(T[1]) * D(z2)));
}

// rotation part of pointAssociateToMap, precomputed once per pose: cos/sin of T[0..2] in double
struct MapRot { double c0, s0, c1, s1, c2, s2; float t3, t4, t5; };
LOAM_HD MapRot map_rot(const float* T) {
  MapRot r;
  r.c0 = dcos(T[0]); r.s0 = dsin(T[0]);
  r.c1 = dcos(T[1]); r.s1 = dsin(T[1]);
  r.c2 = dcos(T[2]); r.s2 = dsin(T[2]);
  r.t3 = T[3]; r.t4 = T[4]; r.t5 = T[5];
  return r;
}
LOAM_HD float4 point_to_map(const MapRot& r, float4 pi) {
  float x1 = (float)(r.c2 * D(pi.x) - r.s2 * D(pi.y));
  float y1 = (float)(r.s2 * D(pi.x) + r.c2 * D(pi.y));
  float z1 = pi.z;
  float y2 = (float)(r.c0 * D(y1) - r.s0 * D(z1));
  float z2 = (float)(r.s0 * D(y1) + r.c0 * D(z1));
  float4 o;
  o.x = (float)(r.c1 * D(x1) + r.s1 * D(z2) + D(r.t3));
  o.y = y2 + r.t4;
  o.z = (float)(-r.s1 * D(x1) + r.c1 * D(z2) + D(r.t5));
  o.w = pi.w;
  return o;
}
LOAM_HD float4 point_to_tobe_mapped(const MapRot& r, float4 pi) {
  float x1 = (float)(r.c1 * D(pi.x - r.t3) - r.s1 * D(pi.z - r.t5));
  float y1 = pi.y - r.t4;
  float z1 = (float)(r.s1 * D(pi.x - r.t3) + r.c1 * D(pi.z - r.t5));
  float y2 = (float)(r.c0 * D(y1) + r.s0 * D(z1));
  float z2 = (float)(-r.s0 * D(y1) + r.c0 * D(z1));
  float4 o;
  o.x = (float)(r.c2 * D(x1) + r.s2 * D(y2));
  o.y = (float)(-r.s2 * D(x1) + r.c2 * D(y2));
  o.z = z2;
  o.w = pi.w;
  return o;
}

// tf::Quaternion::setRPY and tf::Matrix3x3::getRPY (double)
// (sin and cos of one angle come from one sincos call: GCC -O2 and above merges the pair in tf's
// inlined setRPY, and glibc >= 2.28's sincos differs from separate sin / cos in the last bit of
// ~0.1 % of doubles — the message quaternion is published in double, so that bit is visible)
LOAM_HD void sincos_pair(double x, double& s, double& c) {
#ifdef __HIP_DEVICE_COMPILE__
  sincos(x, &s, &c);
#else
  ::sincos(x, &s, &c);
#endif
}
LOAM_HD void quat_from_rpy(double roll, double pitch, double yaw, double* q) {
  double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
  double cy, sy, cp, sp, cr, sr;
  sincos_pair(hy, sy, cy);
  sincos_pair(hp, sp, cp);
  sincos_pair(hr, sr, cr);
  q[0] = sr * cp * cy - cr * sp * sy;
  q[1] = cr * sp * cy + sr * cp * sy;
  q[2] = cr * cp * sy - sr * sp * cy;
  q[3] = cr * cp * cy + sr * sp * sy;
}
LOAM_HD void rpy_from_quat(const double* q, double& roll, double& pitch, double& yaw) {
  double d = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  double s = 2.0 / d;
  double xs = q[0] * s, ys = q[1] * s, zs = q[2] * s;
  double wx = q[3] * xs, wy = q[3] * ys, wz = q[3] * zs;
  double xx = q[0] * xs, xy = q[0] * ys, xz = q[0] * zs;
  double yy = q[1] * ys, yz = q[1] * zs, zz = q[2] * zs;
  double m00 = 1.0 - (yy + zz), m02 = xz + wy, m10 = xy + wz;
  double m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
  if (fabs(m20) >= 1) {
    yaw = 0;
    double delta = atan2(m00, m02);
    if (m20 > 0) { pitch = M_PI / 2.0; roll = pitch + delta; }
    else { pitch = -M_PI / 2.0; roll = -pitch + delta; }
  } else {
    pitch = -asin(m20);
    roll = atan2(m21 / cos(pitch), m22 / cos(pitch));
    yaw = atan2(m10 / cos(pitch), m00 / cos(pitch));
  }
}
// odometry transformSum -> nav_msgs orientation -> receiving node's transformSum
LOAM_HD void pose_through_msg(const float* in, float* out) {
  double g[4];
  quat_from_rpy(D(in[2]), -D(in[0]), -D(in[1]), g);
  double msg[4] = {-g[1], -g[2], g[0], g[3]};
  double back[4] = {msg[2], -msg[0], -msg[1], msg[3]};
  double roll, pitch, yaw;
  rpy_from_quat(back, roll, pitch, yaw);
  out[0] = (float)(-pitch);
  out[1] = (float)(-yaw);
  out[2] = (float)roll;
  out[3] = in[3]; out[4] = in[4]; out[5] = in[5];
}

}  // namespace loampose

#endif
