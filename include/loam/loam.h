/* loam.h — C-ABI of the MI355X LOAM scan-matching engine (libloam_hip.so).
 *
 * Drop-in for the compute bodies of the four ROS nodes of the reference
 * (/root/reference = Maofei/loam_velodyne-1).  Each entry point replaces one node callback:
 *
 *   loam_scan_registration  <- laserCloudHandler        src/scanRegistration.cpp:211-636
 *   loam_imu                <- imuHandler               src/scanRegistration.cpp:638-660 and
 *                              laserMapping imuHandler  src/laserMapping.cpp:323-335
 *   loam_odometry           <- laserOdometry loop body  src/laserOdometry.cpp:413-931
 *                              (inputs = what handlers :275-354 store)
 *   loam_mapping            <- laserMapping loop body   src/laserMapping.cpp:411-1097
 *                              (inputs = what handlers :274-321 store)
 *   loam_mapping_surround   <- /laser_cloud_surround    src/laserMapping.cpp:1038-1058
 *   loam_maintenance        <- transformMaintenance     src/transformMaintenance.cpp:147-203
 *   loam_batch_*            <- config 4 of BASELINE.json (independent problems, no reference
 *                              equivalent: one problem = the bodies above composed)
 *
 * Conventions: no C++ types cross the boundary; all host storage is caller-owned and never
 * retained after a call; a context owns its device memory, one HIP device and its HIP streams
 * (the node bodies run on one; a batch step spreads over up to four, loam_batch_sync drains them
 * all); a context is not thread-safe, distinct contexts may run concurrently.  Every function returns
 * LOAM_OK (0) or a negative LOAM_E_* code; loam_last_error() describes the last failure on the
 * calling thread.  LOAM_E_CAPACITY writes the required size back into the cloud's `count`.
 */
#ifndef LOAM_LOAM_H
#define LOAM_LOAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LOAM_OK 0
#define LOAM_E_INVAL (-1)
#define LOAM_E_CAPACITY (-2)
#define LOAM_E_HIP (-3)
#define LOAM_E_NOT_READY (-4) /* scan registration inside systemDelay (Q1) */
#define LOAM_E_NOMEM (-5)

/* published-flag bits of loam_odometry (the topics laserOdometry publishes on this call) */
#define LOAM_PUB_POSE 1   /* /laser_odom_to_init  (src/laserOdometry.cpp:858-873) */
#define LOAM_PUB_CLOUDS 2 /* /laser_cloud_corner_last + /laser_cloud_surf_last (:439-449, :913-923) */
#define LOAM_PUB_FULL 4   /* /velodyne_cloud_3    (:925-929) */

/* ring-ID models for scan registration */
#define LOAM_RING_VLP16 0  /* reference: round(angle) -> r>0 ? r : r+(N-1)  src/scanRegistration.cpp:248-260 */
#define LOAM_RING_LINEAR 1 /* bk HDL-64E hint: int((angle-lo)/step + 0.5f), bk src/scanRegistration.cpp:268-275 */

/* PCL PointXYZI payload in a 16-byte record (PCL's in-memory PointXYZI is 32 B with padding).
 * intensity = ring + 0.1*relTime out of scan registration (src/scanRegistration.cpp:283-284),
 * the integer ring after TransformToEnd (src/laserOdometry.cpp:193). */
typedef struct { float x, y, z, intensity; } loam_point;

/* the reference's float transform[6] layout: (rx, ry, rz, tx, ty, tz) in the camera frame
 * (x left, y up, z forward), e.g. transformSum src/laserOdometry.cpp:94 */
typedef struct { float rx, ry, rz, tx, ty, tz; } loam_pose6;

/* caller-owned input cloud; x, y, z floats at byte offsets 0, 4, 8 of each record
 * (accepts 16-B PointXYZ/loam_point and 32-B PointXYZI / velodyne XYZIR records); stride_bytes a
 * multiple of 4, data at any alignment (e.g. a PointCloud2 message's own buffer, loam_pc2_cloud) */
typedef struct { const void *data; uint32_t count; uint32_t stride_bytes; } loam_cloud_in;

/* caller-owned output storage; count = points written (or required, on LOAM_E_CAPACITY) */
typedef struct { loam_point *pts; uint32_t count; uint32_t capacity; } loam_cloud_out;

/* the six topics scanRegistration publishes (src/scanRegistration.cpp:584-635) */
typedef struct {
  loam_cloud_out full;       /* /velodyne_cloud_2 */
  loam_cloud_out sharp;      /* /laser_cloud_sharp */
  loam_cloud_out less_sharp; /* /laser_cloud_less_sharp */
  loam_cloud_out flat;       /* /laser_cloud_flat */
  loam_cloud_out less_flat;  /* /laser_cloud_less_flat */
  float imu_trans[12];       /* /imu_trans: start RPY, cur RPY, shift, velo (zeros without IMU) */
} loam_features;

typedef struct {
  uint32_t n_rings;        /* N_SCANS (16)                                  scanRegistration.cpp:61 */
  uint32_t ring_model;     /* LOAM_RING_VLP16 | LOAM_RING_LINEAR */
  float ring_lo_deg;       /* LOAM_RING_LINEAR lower bound (-24.8) */
  float ring_hi_deg;       /* LOAM_RING_LINEAR upper bound (2.0) */
  uint32_t system_delay;   /* 20                                            scanRegistration.cpp:57 */
  uint32_t max_points;     /* per-sweep capacity (40000 in the reference)   scanRegistration.cpp:63 */
  uint32_t od_max_iter;    /* 25                                            laserOdometry.cpp:470 */
  uint32_t mp_max_iter;    /* 10                                            laserMapping.cpp:710 */
  uint32_t skip_frame_num; /* 1                                             laserOdometry.cpp:51 */
  uint32_t map_capacity;   /* device map-store capacity in points (per map instance) */
} loam_config;

/* per-call counters; feed the algorithmic-byte formula of SURVEY.md §8(d) */
typedef struct {
  uint64_t n_raw, n_ring;                       /* SR input points, ring-sorted points */
  uint64_t n_sharp, n_less_sharp, n_flat, n_less_flat;
  uint64_t od_iters, od_assoc_rounds, od_rows_sum, od_corner_last, od_surf_last, od_queries;
  uint64_t od_assoc_points;                     /* sum over problems of rounds x (C + S) */
  uint64_t mp_iters, mp_rows_sum, mp_stack, mp_map_points, mp_map_valid_points;
  uint64_t mp_stack_iters;                      /* sum over problems of iterations x stack size */
  uint64_t mp_fits;                             /* line / plane fits computed (the rest reused: same ordered 5-NN) */
  uint64_t od_query_iters;                      /* sum over problems of L-M iterations x queries (sharp + flat) */
  uint64_t od_row_evals;                        /* Jacobian rows evaluated: sum of queries x it(it+1)/2 (Q12) */
  uint64_t bytes_sr, bytes_od, bytes_mp;        /* algorithmic bytes, SURVEY.md §8(d) */
  double ms_sr, ms_od, ms_mp;                   /* device time per stage (HIP events) */
  /* reference branches taken (batch: summed over problems) */
  uint64_t od_degenerate_steps; /* odometry L-M updates projected by the iteration-0 degeneracy
                                   analysis (src/laserOdometry.cpp:770-797, Q15) */
  uint64_t od_nan_skips;        /* odometry L-M updates skipped by the NaN guard (:799-811, Q16) */
  uint64_t mp_degenerate_steps; /* mapping L-M updates projected (src/laserMapping.cpp:927-954) */
  uint64_t mp_grid_shifts;      /* cube-grid slab shifts of the recentring (:454-614, Q23) */
  /* memory work the search kernels actually did (the bench's gathered-byte roofline) */
  uint64_t mp_nn_candidates;    /* map points whose distance the 5-NN evaluated (incl. the seeds) */
  uint64_t mp_nn_cells;         /* hash bucket ranges the 5-NN read */
  uint64_t od_assoc_gathered;   /* Last-cloud points the association loaded (cells, fallback, windows) */
  uint64_t od_assoc_boxes;      /* 64-point chunk boxes the association loaded */
} loam_stats;

typedef struct loam_ctx loam_ctx;

void loam_config_default(loam_config *cfg);               /* reference constants (VLP-16) */
int loam_create(loam_ctx **out, const loam_config *cfg, int device);
void loam_destroy(loam_ctx *ctx);
const char *loam_last_error(void);

/* = the /imu/data handlers of scanRegistration (src/scanRegistration.cpp:638-660: queue entry, gravity
 * removal, AccumulateIMUShift) and laserMapping (src/laserMapping.cpp:323-335).  quat_xyzw = the
 * sensor_msgs/Imu orientation (x, y, z, w), lin_acc_xyz = linear_acceleration, both float64 as in the
 * message.  Stamps must be non-decreasing (LOAM_E_INVAL otherwise).  With IMU data, scan registration
 * de-skews each point with it (:286-349) and fills imu_trans; odometry and mapping use it through
 * imu_trans and the mapping queue (src/laserOdometry.cpp:330-351, src/laserMapping.cpp:199-226). */
int loam_imu(loam_ctx *ctx, double stamp, const double quat_xyzw[4], const double lin_acc_xyz[3]);

/* = laserCloudHandler.  Returns LOAM_E_NOT_READY for the first system_delay sweeps (Q1). */
int loam_scan_registration(loam_ctx *ctx, double stamp, loam_cloud_in raw, loam_features *out);

/* = laserOdometry loop body for one synchronised set of the six scanRegistration topics.
 * sum_out receives transformSum when LOAM_PUB_POSE is set; the three clouds are written when
 * their flag is set in *published. */
int loam_odometry(loam_ctx *ctx, double stamp, const loam_features *in, loam_pose6 *sum_out,
                  loam_cloud_out *corner_last, loam_cloud_out *surf_last, loam_cloud_out *full_end,
                  int *published);

/* = laserMapping loop body for one synchronised (corner_last, surf_last, full, odometry) set.
 * odom_sum goes through the reference's nav_msgs quaternion round trip.  aft / bef are
 * transformAftMapped / transformBefMapped (the Bef pose the reference smuggles in the twist
 * fields, src/laserMapping.cpp:1082-1087); registered = full cloud in the map frame. */
int loam_mapping(loam_ctx *ctx, double stamp, const loam_pose6 *odom_sum,
                 const loam_cloud_out *corner_last, const loam_cloud_out *surf_last,
                 const loam_cloud_out *full_end, loam_pose6 *aft, loam_pose6 *bef,
                 loam_cloud_out *registered);

/* = the /laser_cloud_surround publish of the laserMapping loop body (src/laserMapping.cpp:1038-1058,
 * mapFrameNum = 5, :52, :405): the map store's 5x5x5 cube neighbourhood of the last mapping frame
 * (laserCloudSurroundInd, :617-670), corner then surf points per cube, VoxelGrid 0.2.  The
 * reference publishes it on the 1st successful loam_mapping frame and every 5th after it: on
 * those frames *published = 1 and out is filled; otherwise *published = 0 and out->count = 0.
 * Call between a loam_mapping and the next (the cloud is computed on demand from the store that
 * frame left; a LOAM_E_CAPACITY call may be repeated with more capacity). */
int loam_mapping_surround(loam_ctx *ctx, loam_cloud_out *out, int *published);

/* ---- device-resident node chain (no reference equivalent: the reference's nodes exchange ROS
 * messages; this is the intra-process / nodelet deployment of the same three bodies) ----
 * One sweep through loam_scan_registration -> loam_odometry -> loam_mapping (on the frames odometry
 * publishes all three clouds, as the node graph does) on one context, the intermediate topics left
 * in device memory: odometry reads scan registration's output buffers in place, mapping reads
 * odometry's published CornerLast / SurfLast / full-end buffers in place.  Same kernels, same values
 * as the three message calls; loam_mapping_surround works after it as after loam_mapping.
 * Returns LOAM_E_NOT_READY inside system_delay.  registered: capacity 0 = not downloaded.
 * (Tuning stream_defer, default on, for this call: the bookkeeping only the next sweep reads —
 * mapping's map update, odometry's hash tables of the new Last clouds — runs on the context's second
 * stream after the call has its results; the next call waits for it on the device.  A map-update
 * capacity error is then reported by the next call.) */
typedef struct {
  int32_t published;          /* loam_odometry's LOAM_PUB_* flags for this sweep */
  int32_t mapped;             /* 1 when laserMapping ran on this sweep */
  loam_pose6 od_sum;          /* /laser_odom_to_init (transformSum), when LOAM_PUB_POSE */
  loam_pose6 aft, bef;        /* transformAftMapped / transformBefMapped, when mapped */
  loam_cloud_out registered;  /* /velodyne_cloud_registered, when mapped and capacity > 0 */
} loam_chain_out;
int loam_chain_sweep(loam_ctx *ctx, double stamp, loam_cloud_in raw, loam_chain_out *out);

/* = transformMaintenance laserOdometryHandler with the last odomAftMappedHandler state.
 * Pure host function (scalar pose algebra, no kernel). */
int loam_maintenance(const loam_pose6 *odom_sum, const loam_pose6 *bef, const loam_pose6 *aft,
                     loam_pose6 *integrated);

/* ---- batched independent problems (config 4) ----
 * problem i = scan registration of (prev_i, cur_i), odometry seeded from prev_i and solved on
 * cur_i, mapping of prev_i into an empty map then solved for cur_i.
 * upload copies the host sweeps into device memory; run executes every problem on the device
 * with all inputs resident in HBM; download copies the poses back.  run only enqueues: for
 * n >= 64 (tunings step_pipe / sr_ahead) consecutive runs overlap as a software pipeline — a run's
 * odometry beside the previous run's mapping, the next run's scan registration and odometry seed
 * enqueued ahead (they re-run the same uploaded problems, unless loam_batch_feed supplies each run's
 * sweeps) — and sync waits for all of it.  download returns the last run's results. */
int loam_batch_upload(loam_ctx *ctx, uint32_t n, const loam_cloud_in *prev,
                      const loam_cloud_in *cur);
int loam_batch_run(loam_ctx *ctx);
/* the sweeps of the NEXT loam_batch_run: n independent problems of the uploaded batch size (a new
 * batch arriving over time).  In the step pipeline (n >= tuning step_pipe) the sweeps are copied from
 * pinned staging into the scan-registration set that step reads, on the pipeline's own stream behind
 * that set's previous reader, and that step's scan registration + odometry seed are enqueued there
 * at once, so fresh batches overlap the running steps; a fed context no longer re-runs the resident
 * sweeps ahead (a run without a feed re-runs that set's last sweeps).  Otherwise (sequential steps)
 * the same as loam_batch_upload.  The call packs the sweeps on the calling thread and returns once
 * the copies are enqueued; the caller's buffers are free on return. */
int loam_batch_feed(loam_ctx *ctx, uint32_t n, const loam_cloud_in *prev, const loam_cloud_in *cur);
int loam_batch_sync(loam_ctx *ctx);   /* waits for the work enqueued by loam_batch_run */
int loam_batch_download(loam_ctx *ctx, loam_pose6 *od_sum, loam_pose6 *aft, loam_stats *stats);
/* per-problem L-M results of the last run behind loam_batch_download's poses, for parity checks
 * (any pointer may be NULL): the odometry and mapping iteration counts (the convergence decisions)
 * and the odometry's solved increment transform[6] (src/laserOdometry.cpp:93, :811; the pose the
 * accumulation and TransformToEnd use) */
int loam_batch_lm_info(loam_ctx *ctx, int32_t *od_iters, int32_t *mp_iters, loam_pose6 *od_transform);

/* scheduling (no reference equivalent; the reference's nodes are OS processes): priority of the
 * context's HIP streams.  priority > 0 = the device's highest stream priority, 0 = normal,
 * < 0 = lowest.  Used by a node pipeline to favour its critical node (laserMapping) when several
 * contexts share one GPU.  Waits for the context's queued work, then replaces its streams. */
int loam_set_stream_priority(loam_ctx *ctx, int priority);

/* launch-shape choices of the batch / streaming L-M loops by batch size (no reference equivalent):
 * key = one of od_small_max, od_fused_max, mp_small_max, mp_fused_max, od_assoc_wg, fit_wg, graph,
 * vg_merge, vg_merge_min, vg_split, sr_ahead, sr_ahead_at, step_pipe, batch_streams, pipe_mp_sets, od_sel_min, od_win_mono,
 * od_win_mono_min, od_moments_min, od_persist, mp_persist, stream_defer, od_graph, pipe_sr_sets (loam_velodyne-1_amd/csrc/engine.hpp,
 * struct Tuning).  Every choice computes the same results bit for bit except od_moments_min (the odometry's
 * stored rows as per-query fp64 moments: within the north star's 1e-4 of the reference);
 * the defaults are the measured fastest.  LOAM_E_INVAL for an unknown key or a value out of range.
 * Takes effect from the next call (waits for the context's queued work). */
int loam_set_tuning(loam_ctx *ctx, const char *key, long long value);
/* the current value of a launch choice (LOAM_E_INVAL for an unknown key) */
int loam_get_tuning(loam_ctx *ctx, const char *key, long long *value);

/* last-call statistics of a context (stage device times, counts, algorithmic bytes) */
int loam_get_stats(loam_ctx *ctx, loam_stats *stats);

/* diagnostics (no reference equivalent): per-kernel device time of the batch path, measured with
 * HIP events on the context stream.  loam_get_kernel_times writes "name total_ms launches\n" lines. */
int loam_set_profiling(loam_ctx *ctx, int on);
int loam_get_kernel_times(loam_ctx *ctx, char *buf, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* LOAM_LOAM_H */
