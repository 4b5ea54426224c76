/* loam_bag.h — recorded-sweep ingest for the MI355X LOAM engine (libloam_hip.so), host only.
 *
 * The reference reads its input from ROS topics: /velodyne_points (sensor_msgs/PointCloud2,
 * converted by pcl::fromROSMsg, src/scanRegistration.cpp:225-226) and /imu/data (sensor_msgs/Imu,
 * src/scanRegistration.cpp:638-660), fed by `rosbag play` of the datasets its README names
 * (nsh_indoor_outdoor.bag ...).  This header replaces that ingest without ROS:
 *
 *   loam_bag_*      a rosbag v2.0 reader (records, chunks uncompressed / bz2 / lz4, connection
 *                   records) that yields the messages in file order, as `rosbag play` publishes them;
 *   loam_pc2_*      sensor_msgs/PointCloud2 wire format: header stamp, fields by name (x, y, z,
 *                   intensity, ring), point_step, is_dense; the cloud handed to
 *                   loam_scan_registration without a copy when x, y, z sit at offsets 0/4/8
 *                   (velodyne PointXYZIR, PCL PointXYZ/PointXYZI), packed otherwise;
 *   loam_imu_parse  sensor_msgs/Imu: header stamp, orientation, linear acceleration — the
 *                   arguments of loam_imu.
 *
 * Same conventions as loam.h: caller-owned storage, LOAM_OK / negative LOAM_E_* codes,
 * loam_last_error() for the message.  A bag handle is not thread-safe.  bz2 / lz4 chunks use the
 * system libbz2.so.1 / liblz4.so.1 (loaded on first use; LOAM_E_INVAL if absent).
 */
#ifndef LOAM_LOAM_BAG_H
#define LOAM_LOAM_BAG_H

#include <stdint.h>

#include "loam.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LOAM_BAG_END 1 /* loam_bag_next: no more messages */

typedef struct loam_bag loam_bag;

typedef struct {
  const char *topic;   /* connection topic; valid while the bag is open */
  const char *type;    /* message type, e.g. "sensor_msgs/PointCloud2"; valid while the bag is open */
  double stamp;        /* record (receive) time, seconds */
  const uint8_t *data; /* serialized message; valid until the next loam_bag_next / loam_bag_close */
  uint32_t size;
} loam_bag_msg;

int loam_bag_open(loam_bag **out, const char *path);
void loam_bag_close(loam_bag *bag);
/* the next message record in file order: LOAM_OK, LOAM_BAG_END, or a negative error */
int loam_bag_next(loam_bag *bag, loam_bag_msg *msg);

typedef struct {
  double stamp;                     /* header.stamp, seconds */
  uint32_t width, height;
  uint32_t point_step, row_step;
  int32_t off_x, off_y, off_z;      /* FLOAT32 field offsets (required) */
  int32_t off_intensity, off_ring;  /* -1 when absent */
  uint8_t is_bigendian, is_dense;
  const uint8_t *data;              /* points (into the message buffer) */
  uint32_t data_size;
} loam_pc2;

/* parses a serialized sensor_msgs/PointCloud2 (ROS1 wire format); LOAM_E_INVAL on a malformed
 * message, a big-endian cloud or x / y / z fields that are not FLOAT32 */
int loam_pc2_parse(const uint8_t *msg, uint32_t size, loam_pc2 *out);

/* the cloud as loam_scan_registration reads it (x, y, z floats at offsets 0 / 4 / 8 of each
 * record): the message's own points when the layout already is that (no copy), else x, y, z
 * packed into scratch (capacity scratch_cap points; LOAM_E_CAPACITY with the required count in
 * out->count otherwise).  The points stay valid as long as the message / scratch does; in place,
 * they are at whatever alignment the message gives them. */
int loam_pc2_cloud(const loam_pc2 *pc, loam_point *scratch, uint32_t scratch_cap, loam_cloud_in *out);

/* parses a serialized sensor_msgs/Imu: header.stamp, orientation (x, y, z, w), linear_acceleration */
int loam_imu_parse(const uint8_t *msg, uint32_t size, double *stamp, double quat_xyzw[4], double lin_acc_xyz[3]);

#ifdef __cplusplus
}
#endif

#endif
