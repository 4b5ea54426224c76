/* loam_msg.h — the reference's ROS message conventions for poses, without ROS (libloam_hip.so).
 *
 * The four reference nodes exchange poses as nav_msgs/Odometry and tf transforms with an axis
 * permutation and, on /aft_mapped_to_init, transformBefMapped smuggled through the twist fields.
 * A ROS wrapper over loam.h fills and reads its messages with these two functions, so that the
 * unchanged downstream nodes and RViz see exactly what the reference publishes:
 *
 *   loam_msg_from_pose  <- laserOdometry.cpp:858-873   (/laser_odom_to_init, tf /laser_odom)
 *                          laserMapping.cpp:1071-1094  (/aft_mapped_to_init + Bef in the twist, tf /aft_mapped)
 *                          transformMaintenance.cpp:163-178 (/integrated_to_init, tf /camera)
 *   loam_pose_from_msg  <- laserMapping.cpp:304-321    (laserOdometryHandler)
 *                          transformMaintenance.cpp:147-160, 182-203 (both handlers)
 *
 * Arithmetic as in the reference: tf::createQuaternionMsgFromRollPitchYaw(rz, -rx, -ry) and
 * tf::Matrix3x3::getRPY in double (tfScalar), float pose values widened on assignment and
 * narrowed back on reading.  Pure host functions: no device, no context.
 */
#ifndef LOAM_MSG_H
#define LOAM_MSG_H

#include <stdint.h>

#include "loam.h"

#ifdef __cplusplus
extern "C" {
#endif

/* which of the reference's three pose topics a message is */
#define LOAM_MSG_LASER_ODOM 0 /* /laser_odom_to_init, "/camera_init" -> "/laser_odom"  (laserOdometry.cpp:391-397) */
#define LOAM_MSG_AFT_MAPPED 1 /* /aft_mapped_to_init, "/camera_init" -> "/aft_mapped"  (laserMapping.cpp:364-370) */
#define LOAM_MSG_INTEGRATED 2 /* /integrated_to_init, "/camera_init" -> "/camera" (transformMaintenance.cpp:218-224) */

/* the fields of nav_msgs/Odometry the reference writes (all float64 in the message) */
typedef struct {
  double stamp;              /* header.stamp, seconds */
  const char *frame_id;      /* header.frame_id (static string) */
  const char *child_frame_id;
  double orientation[4];     /* pose.pose.orientation x, y, z, w */
  double position[3];        /* pose.pose.position x, y, z */
  double twist_angular[3];   /* twist.twist.angular: transformBefMapped rx, ry, rz (AFT_MAPPED), else 0 */
  double twist_linear[3];    /* twist.twist.linear: transformBefMapped tx, ty, tz (AFT_MAPPED), else 0 */
} loam_odometry_msg;

/* the payload of the tf::StampedTransform broadcast beside each message */
typedef struct {
  double stamp;
  const char *frame_id, *child_frame_id;
  double rotation[4];        /* tf::Quaternion x, y, z, w */
  double origin[3];
} loam_tf_msg;

/* pose (and, for LOAM_MSG_AFT_MAPPED, bef) -> message and tf transform; tf may be NULL.
 * LOAM_E_INVAL on a bad kind, a NULL pose / msg, or a NULL bef with LOAM_MSG_AFT_MAPPED. */
int loam_msg_from_pose(int kind, double stamp, const loam_pose6 *pose, const loam_pose6 *bef,
                       loam_odometry_msg *msg, loam_tf_msg *tf);

/* message -> pose as the receiving handlers read it; bef (may be NULL) <- the twist fields. */
int loam_pose_from_msg(const loam_odometry_msg *msg, loam_pose6 *pose, loam_pose6 *bef);

#ifdef __cplusplus
}
#endif
#endif /* LOAM_MSG_H */
