// The reference's pose message conventions (include/loam/loam_msg.h): host functions over the
// tf algebra of pose_math.hpp.
#include <cstring>
#include <string>

#include "../../include/loam/loam_msg.h"
#include "engine.hpp"
#include "pose_math.hpp"

using loamdev::D;

namespace {

struct Frames {
  const char *frame, *child;
};

const Frames kFrames[3] = {{"/camera_init", "/laser_odom"},   // laserOdometry.cpp:391-397
                           {"/camera_init", "/aft_mapped"},   // laserMapping.cpp:364-370
                           {"/camera_init", "/camera"}};      // transformMaintenance.cpp:218-224

}  // namespace

extern "C" {

int loam_msg_from_pose(int kind, double stamp, const loam_pose6* pose, const loam_pose6* bef,
                       loam_odometry_msg* msg, loam_tf_msg* tf) {
  if (kind < LOAM_MSG_LASER_ODOM || kind > LOAM_MSG_INTEGRATED || !pose || !msg ||
      (kind == LOAM_MSG_AFT_MAPPED && !bef)) {
    loam::set_last_error("loam_msg_from_pose: bad kind or null argument");
    return LOAM_E_INVAL;
  }
  const float* p = (const float*)pose;
  // geoQuat = createQuaternionMsgFromRollPitchYaw(rz, -rx, -ry) (laserOdometry.cpp:858,
  // laserMapping.cpp:1071-1072, transformMaintenance.cpp:163-164)
  double g[4];
  loampose::quat_from_rpy(D(p[2]), -D(p[0]), -D(p[1]), g);
  std::memset(msg, 0, sizeof(*msg));
  msg->stamp = stamp;
  msg->frame_id = kFrames[kind].frame;
  msg->child_frame_id = kFrames[kind].child;
  // orientation = (-q.y, -q.z, q.x, q.w), position = translation (laserOdometry.cpp:860-866)
  msg->orientation[0] = -g[1];
  msg->orientation[1] = -g[2];
  msg->orientation[2] = g[0];
  msg->orientation[3] = g[3];
  for (int i = 0; i < 3; ++i) msg->position[i] = D(p[3 + i]);
  if (kind == LOAM_MSG_AFT_MAPPED) {  // transformBefMapped in the twist (laserMapping.cpp:1082-1087)
    const float* b = (const float*)bef;
    for (int i = 0; i < 3; ++i) {
      msg->twist_angular[i] = D(b[i]);
      msg->twist_linear[i] = D(b[3 + i]);
    }
  }
  if (tf) {  // setRotation(Quaternion(-q.y, -q.z, q.x, q.w)), setOrigin(translation) (:870-872)
    tf->stamp = stamp;
    tf->frame_id = msg->frame_id;
    tf->child_frame_id = msg->child_frame_id;
    for (int i = 0; i < 4; ++i) tf->rotation[i] = msg->orientation[i];
    for (int i = 0; i < 3; ++i) tf->origin[i] = msg->position[i];
  }
  return LOAM_OK;
}

int loam_pose_from_msg(const loam_odometry_msg* msg, loam_pose6* pose, loam_pose6* bef) {
  if (!msg || !pose) {
    loam::set_last_error("loam_pose_from_msg: null argument");
    return LOAM_E_INVAL;
  }
  // Matrix3x3(Quaternion(q.z, -q.x, -q.y, q.w)).getRPY(roll, pitch, yaw); pose = (-pitch, -yaw,
  // roll, position) (laserMapping.cpp:308-318, transformMaintenance.cpp:149-159, 184-194)
  const double q[4] = {msg->orientation[2], -msg->orientation[0], -msg->orientation[1], msg->orientation[3]};
  double roll, pitch, yaw;
  loampose::rpy_from_quat(q, roll, pitch, yaw);
  float* p = (float*)pose;
  p[0] = (float)(-pitch);
  p[1] = (float)(-yaw);
  p[2] = (float)roll;
  for (int i = 0; i < 3; ++i) p[3 + i] = (float)msg->position[i];
  if (bef) {  // transformMaintenance.cpp:196-202
    float* b = (float*)bef;
    for (int i = 0; i < 3; ++i) {
      b[i] = (float)msg->twist_angular[i];
      b[3 + i] = (float)msg->twist_linear[i];
    }
  }
  return LOAM_OK;
}

}  // extern "C"
