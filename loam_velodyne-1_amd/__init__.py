"""ctypes binding of libloam_hip.so, the MI355X LOAM scan-matching engine (C-ABI in
include/loam/loam.h).  One `Engine` = one loam_ctx = the four reference ROS nodes' compute bodies
on one GPU:

    scan_registration(raw)          laserCloudHandler    src/scanRegistration.cpp:211-636
    odometry(features)              laserOdometry body   src/laserOdometry.cpp:413-931
    mapping(pose, corner, surf, full) laserMapping body  src/laserMapping.cpp:411-1097
    maintenance(sum, bef, aft)      transformMaintenance src/transformMaintenance.cpp:147-203
    batch_*                         config 4 (independent problems)

There is no CPU path: without a GPU (or without the built library) every call raises.
The package directory name contains '-', so import it with
importlib.import_module("loam_velodyne-1_amd")."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LOAM_HIP_LIB") or os.path.join(_HERE, "libloam_hip.so")
_LIB = None

LOAM_OK, LOAM_E_INVAL, LOAM_E_CAPACITY, LOAM_E_HIP, LOAM_E_NOT_READY, LOAM_E_NOMEM = 0, -1, -2, -3, -4, -5
PUB_POSE, PUB_CLOUDS, PUB_FULL = 1, 2, 4
RING_VLP16, RING_LINEAR = 0, 1


class LoamError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"loam error {code}: {msg}")
        self.code = code


class CloudIn(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("count", ctypes.c_uint32), ("stride_bytes", ctypes.c_uint32)]


class CloudOut(ctypes.Structure):
    _fields_ = [("pts", ctypes.c_void_p), ("count", ctypes.c_uint32), ("capacity", ctypes.c_uint32)]


class Features(ctypes.Structure):
    _fields_ = [("full", CloudOut), ("sharp", CloudOut), ("less_sharp", CloudOut),
                ("flat", CloudOut), ("less_flat", CloudOut), ("imu_trans", ctypes.c_float * 12)]


class Pose6(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("rx", "ry", "rz", "tx", "ty", "tz")]

    def arr(self):
        return np.array([self.rx, self.ry, self.rz, self.tx, self.ty, self.tz], np.float32)

    @staticmethod
    def of(a):
        p = Pose6()
        p.rx, p.ry, p.rz, p.tx, p.ty, p.tz = [float(v) for v in a]
        return p


class OdometryMsg(ctypes.Structure):
    """include/loam/loam_msg.h loam_odometry_msg (nav_msgs/Odometry fields the reference writes)"""
    _fields_ = [("stamp", ctypes.c_double), ("frame_id", ctypes.c_char_p), ("child_frame_id", ctypes.c_char_p),
                ("orientation", ctypes.c_double * 4), ("position", ctypes.c_double * 3),
                ("twist_angular", ctypes.c_double * 3), ("twist_linear", ctypes.c_double * 3)]


class TfMsg(ctypes.Structure):
    _fields_ = [("stamp", ctypes.c_double), ("frame_id", ctypes.c_char_p), ("child_frame_id", ctypes.c_char_p),
                ("rotation", ctypes.c_double * 4), ("origin", ctypes.c_double * 3)]


MSG_LASER_ODOM, MSG_AFT_MAPPED, MSG_INTEGRATED = 0, 1, 2


class Config(ctypes.Structure):
    _fields_ = [("n_rings", ctypes.c_uint32), ("ring_model", ctypes.c_uint32),
                ("ring_lo_deg", ctypes.c_float), ("ring_hi_deg", ctypes.c_float),
                ("system_delay", ctypes.c_uint32), ("max_points", ctypes.c_uint32),
                ("od_max_iter", ctypes.c_uint32), ("mp_max_iter", ctypes.c_uint32),
                ("skip_frame_num", ctypes.c_uint32), ("map_capacity", ctypes.c_uint32)]


STAT_U64 = ("n_raw", "n_ring", "n_sharp", "n_less_sharp", "n_flat", "n_less_flat",
            "od_iters", "od_assoc_rounds", "od_rows_sum", "od_corner_last", "od_surf_last", "od_queries",
            "od_assoc_points",
            "mp_iters", "mp_rows_sum", "mp_stack", "mp_map_points", "mp_map_valid_points", "mp_stack_iters",
            "mp_fits", "od_query_iters", "od_row_evals",
            "bytes_sr", "bytes_od", "bytes_mp")


STAT_BRANCH = ("od_degenerate_steps", "od_nan_skips", "mp_degenerate_steps", "mp_grid_shifts")
STAT_WORK = ("mp_nn_candidates", "mp_nn_cells", "od_assoc_gathered", "od_assoc_boxes")


class ChainOut(ctypes.Structure):
    _fields_ = [("published", ctypes.c_int32), ("mapped", ctypes.c_int32), ("od_sum", Pose6),
                ("aft", Pose6), ("bef", Pose6), ("registered", CloudOut)]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in STAT_U64] + \
               [(n, ctypes.c_double) for n in ("ms_sr", "ms_od", "ms_mp")] + \
               [(n, ctypes.c_uint64) for n in STAT_BRANCH + STAT_WORK]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


EXPORTS = ("loam_config_default", "loam_create", "loam_destroy", "loam_last_error", "loam_imu",
           "loam_scan_registration", "loam_odometry", "loam_mapping", "loam_mapping_surround",
           "loam_maintenance", "loam_chain_sweep",
           "loam_batch_upload", "loam_batch_feed", "loam_batch_run", "loam_batch_sync", "loam_batch_download", "loam_batch_lm_info", "loam_get_stats",
           "loam_set_profiling", "loam_get_kernel_times", "loam_set_stream_priority", "loam_set_tuning",
           "loam_get_tuning",
           # include/loam/loam_bag.h: recorded-sweep ingest (rosbag v2, PointCloud2, Imu)
           "loam_bag_open", "loam_bag_close", "loam_bag_next", "loam_pc2_parse", "loam_pc2_cloud",
           "loam_imu_parse",
           # include/loam/loam_msg.h: the reference's pose message conventions
           "loam_msg_from_pose", "loam_pose_from_msg")


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        P, PP = ctypes.POINTER, ctypes.c_void_p
        L.loam_config_default.argtypes = [P(Config)]
        L.loam_create.argtypes = [P(PP), P(Config), ctypes.c_int]
        L.loam_destroy.argtypes = [PP]
        L.loam_last_error.restype = ctypes.c_char_p
        L.loam_scan_registration.argtypes = [PP, ctypes.c_double, CloudIn, P(Features)]
        L.loam_imu.argtypes = [PP, ctypes.c_double, P(ctypes.c_double), P(ctypes.c_double)]
        L.loam_odometry.argtypes = [PP, ctypes.c_double, P(Features), P(Pose6), P(CloudOut), P(CloudOut),
                                    P(CloudOut), P(ctypes.c_int)]
        L.loam_mapping.argtypes = [PP, ctypes.c_double, P(Pose6), P(CloudOut), P(CloudOut), P(CloudOut),
                                   P(Pose6), P(Pose6), P(CloudOut)]
        L.loam_mapping_surround.argtypes = [PP, P(CloudOut), P(ctypes.c_int)]
        L.loam_chain_sweep.argtypes = [PP, ctypes.c_double, CloudIn, P(ChainOut)]
        L.loam_maintenance.argtypes = [P(Pose6)] * 4
        L.loam_batch_upload.argtypes = [PP, ctypes.c_uint32, P(CloudIn), P(CloudIn)]
        L.loam_batch_feed.argtypes = [PP, ctypes.c_uint32, P(CloudIn), P(CloudIn)]
        L.loam_batch_run.argtypes = [PP]
        L.loam_batch_sync.argtypes = [PP]
        L.loam_set_profiling.argtypes = [PP, ctypes.c_int]
        L.loam_set_stream_priority.argtypes = [PP, ctypes.c_int]
        L.loam_set_tuning.argtypes = [PP, ctypes.c_char_p, ctypes.c_longlong]
        L.loam_get_tuning.argtypes = [PP, ctypes.c_char_p, P(ctypes.c_longlong)]
        L.loam_get_kernel_times.argtypes = [PP, ctypes.c_char_p, ctypes.c_uint32]
        L.loam_batch_download.argtypes = [PP, P(Pose6), P(Pose6), P(Stats)]
        L.loam_batch_lm_info.argtypes = [PP, P(ctypes.c_int32), P(ctypes.c_int32), P(Pose6)]
        L.loam_get_stats.argtypes = [PP, P(Stats)]
        L.loam_msg_from_pose.argtypes = [ctypes.c_int, ctypes.c_double, P(Pose6), P(Pose6), P(OdometryMsg), P(TfMsg)]
        L.loam_pose_from_msg.argtypes = [P(OdometryMsg), P(Pose6), P(Pose6)]
        _LIB = L
    return _LIB


def _check(rc):
    if rc != LOAM_OK:
        raise LoamError(rc, lib().loam_last_error().decode())
    return rc


def default_config(**kw):
    c = Config()
    lib().loam_config_default(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def _cloud_in(a):
    """an (n, >= 3) float array, or a ready loam_cloud_in (a strided view of caller memory, e.g. a
    PointCloud2 message's records: rosbag.pc2_cloud_in) passed through as is"""
    if isinstance(a, CloudIn):
        return a, None
    a = np.ascontiguousarray(a, np.float32)
    return CloudIn(a.ctypes.data, a.shape[0], a.shape[1] * 4), a


class _Out:
    def __init__(self, cap):
        self.arr = np.empty((max(cap, 1), 4), np.float32)
        self.c = CloudOut(self.arr.ctypes.data, 0, cap)

    def get(self, count=None):
        return self.arr[:self.c.count if count is None else count].copy()


def _cloud_ref(a):
    a = np.ascontiguousarray(a, np.float32).reshape(-1, 4)
    return CloudOut(a.ctypes.data if a.shape[0] else None, a.shape[0], a.shape[0]), a


class Engine:
    # scan_registration / chain_sweep accept a loam_cloud_in view as the raw sweep (rosbag.replay)
    takes_cloud_in = True

    def __init__(self, cfg=None, device=0, cap=None):
        self.cfg = cfg or default_config()
        self.h = ctypes.c_void_p()
        _check(lib().loam_create(ctypes.byref(self.h), ctypes.byref(self.cfg), device))
        self.cap = cap or int(self.cfg.max_points)
        # output storage reused by every call (the results are copied out of it)
        self._sr_outs = [_Out(self.cap) for _ in range(5)]
        self._od_outs = [_Out(self.cap) for _ in range(3)]

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().loam_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        self.close()

    def stats(self):
        s = Stats()
        _check(lib().loam_get_stats(self.h, ctypes.byref(s)))
        return s.as_dict()

    # --- the node bodies
    def imu(self, stamp, quat_xyzw, lin_acc):
        """/imu/data (scanRegistration and laserMapping imuHandlers)"""
        q = (ctypes.c_double * 4)(*[float(v) for v in quat_xyzw])
        a = (ctypes.c_double * 3)(*[float(v) for v in lin_acc])
        _check(lib().loam_imu(self.h, stamp, q, a))

    def scan_registration(self, raw, stamp=0.0):
        ci, keep = _cloud_in(raw)
        outs = self._sr_outs
        f = Features(*[o.c for o in outs])
        rc = lib().loam_scan_registration(self.h, stamp, ci, ctypes.byref(f))
        if rc == LOAM_E_NOT_READY:
            return rc, None
        _check(rc)
        names = ["full", "sharp", "less_sharp", "flat", "less_flat"]
        res = {n: o.get(getattr(f, n).count) for n, o in zip(names, outs)}
        res["imu_trans"] = np.array(f.imu_trans[:], np.float32)
        return 0, res

    def odometry(self, feats, stamp=0.0):
        refs = [_cloud_ref(feats[n]) for n in ("full", "sharp", "less_sharp", "flat", "less_flat")]
        f = Features(*[r[0] for r in refs])
        if "imu_trans" in feats:
            f.imu_trans[:] = [float(v) for v in feats["imu_trans"]]
        pose = Pose6()
        outs = self._od_outs
        for o in outs:
            o.c.count = 0
        pub = ctypes.c_int(0)
        _check(lib().loam_odometry(self.h, stamp, ctypes.byref(f), ctypes.byref(pose), ctypes.byref(outs[0].c),
                                   ctypes.byref(outs[1].c), ctypes.byref(outs[2].c), ctypes.byref(pub)))
        return pub.value, pose.arr(), outs[0].get(), outs[1].get(), outs[2].get()

    def mapping(self, odom_sum, corner, surf, full, stamp=0.0):
        refs = [_cloud_ref(a) for a in (corner, surf, full)]
        aft, bef = Pose6(), Pose6()
        reg = _Out(max(int(np.asarray(full).shape[0]), 1))
        _check(lib().loam_mapping(self.h, stamp, ctypes.byref(Pose6.of(odom_sum)), ctypes.byref(refs[0][0]),
                                  ctypes.byref(refs[1][0]), ctypes.byref(refs[2][0]), ctypes.byref(aft),
                                  ctypes.byref(bef), ctypes.byref(reg.c)))
        return aft.arr(), bef.arr(), reg.get()

    def chain_sweep(self, raw, stamp=0.0, registered=False):
        """one sweep through the three node bodies with the intermediate topics kept on the device
        (loam_chain_sweep): (rc, published, od_sum, aft, bef, registered) -- aft / bef None when
        mapping did not run on this sweep, registered None unless requested"""
        ci, keep = _cloud_in(raw)
        out = ChainOut()
        # (the registered cloud has one point per input point: a CloudIn view carries its count)
        reg = _Out(max(int(ci.count), 1)) if registered else None
        if reg is not None:
            out.registered = reg.c
        rc = lib().loam_chain_sweep(self.h, stamp, ci, ctypes.byref(out))
        if rc == LOAM_E_NOT_READY:
            return rc, 0, None, None, None, None
        _check(rc)
        if not out.mapped:
            return 0, out.published, out.od_sum.arr(), None, None, None
        r = None
        if reg is not None:
            reg.c = out.registered
            r = reg.get()
        return 0, out.published, out.od_sum.arr(), out.aft.arr(), out.bef.arr(), r

    def mapping_surround(self, cap=1 << 16):
        """/laser_cloud_surround of the last mapping frame (laserMapping.cpp:1038-1058): an (n, 4)
        array on the frames the reference publishes it (1st, then every 5th), else None"""
        pub = ctypes.c_int(0)
        out = _Out(cap)
        rc = lib().loam_mapping_surround(self.h, ctypes.byref(out.c), ctypes.byref(pub))
        if rc == LOAM_E_CAPACITY:
            out = _Out(int(out.c.count))
            rc = lib().loam_mapping_surround(self.h, ctypes.byref(out.c), ctypes.byref(pub))
        _check(rc)
        return out.get() if pub.value else None

    # --- config 4
    @staticmethod
    def prepare_batch(prevs, curs):
        """the loam_cloud_in arrays of a batch (kept with the arrays they view), built once for
        repeated batch_feed calls"""
        n = len(prevs)
        keep = []
        a = (CloudIn * n)()
        b = (CloudIn * n)()
        for i in range(n):
            a[i], k1 = _cloud_in(prevs[i])
            b[i], k2 = _cloud_in(curs[i])
            keep += [k1, k2]
        return n, a, b, keep

    def batch_upload(self, prevs, curs):
        n, a, b, _keep = self.prepare_batch(prevs, curs)
        _check(lib().loam_batch_upload(self.h, n, a, b))
        self.n = n

    def batch_feed(self, prevs, curs=None):
        """the sweeps of the next batch_run (loam_batch_feed): (prevs, curs) lists, or a
        prepare_batch result as the only argument"""
        n, a, b, _keep = prevs if curs is None else self.prepare_batch(prevs, curs)
        _check(lib().loam_batch_feed(self.h, n, a, b))

    def batch_run(self):
        _check(lib().loam_batch_run(self.h))

    def sync(self):
        _check(lib().loam_batch_sync(self.h))

    def set_stream_priority(self, priority):
        """> 0 highest, 0 normal, < 0 lowest device stream priority for this context's streams"""
        _check(lib().loam_set_stream_priority(self.h, int(priority)))

    def set_tuning(self, **kv):
        """launch-shape choices by batch size (include/loam/loam.h loam_set_tuning), e.g.
        set_tuning(od_fused_max=0); every choice computes the same results"""
        for k, v in kv.items():
            _check(lib().loam_set_tuning(self.h, k.encode(), int(v)))

    def get_tuning(self, key):
        """the current value of a launch choice (include/loam/loam.h loam_get_tuning)"""
        v = ctypes.c_longlong(0)
        _check(lib().loam_get_tuning(self.h, key.encode(), ctypes.byref(v)))
        return int(v.value)

    def set_profiling(self, on):
        _check(lib().loam_set_profiling(self.h, 1 if on else 0))

    def kernel_times(self):
        """{kernel: (total_ms, launches)} accumulated since profiling was enabled"""
        buf = ctypes.create_string_buffer(1 << 16)
        _check(lib().loam_get_kernel_times(self.h, buf, len(buf)))
        out = {}
        for line in buf.value.decode().splitlines():
            name, ms, n = line.split()
            out[name] = (float(ms), int(n))
        return out

    def batch_download(self):
        od = (Pose6 * self.n)()
        aft = (Pose6 * self.n)()
        st = Stats()
        _check(lib().loam_batch_download(self.h, od, aft, ctypes.byref(st)))
        return (np.array([p.arr() for p in od]), np.array([p.arr() for p in aft]), st.as_dict())

    def batch_lm_info(self):
        """per-problem L-M results of the last run: (odometry iterations, mapping iterations, the
        odometry's solved transform [n, 6])"""
        od = np.zeros(self.n, np.int32)
        mp = np.zeros(self.n, np.int32)
        tr = (Pose6 * self.n)()
        P = ctypes.POINTER(ctypes.c_int32)
        _check(lib().loam_batch_lm_info(self.h, od.ctypes.data_as(P), mp.ctypes.data_as(P), tr))
        return od, mp, np.array([p.arr() for p in tr])


def maintenance(odom_sum, bef, aft):
    out = Pose6()
    _check(lib().loam_maintenance(ctypes.byref(Pose6.of(odom_sum)), ctypes.byref(Pose6.of(bef)),
                                  ctypes.byref(Pose6.of(aft)), ctypes.byref(out)))
    return out.arr()


def msg_from_pose(kind, pose, bef=None, stamp=0.0):
    """pose (+ bef for MSG_AFT_MAPPED) -> (OdometryMsg, TfMsg) as the reference publishes them"""
    m, t = OdometryMsg(), TfMsg()
    b = ctypes.byref(Pose6.of(bef)) if bef is not None else None
    _check(lib().loam_msg_from_pose(kind, stamp, ctypes.byref(Pose6.of(pose)), b, ctypes.byref(m), ctypes.byref(t)))
    return m, t


def pose_from_msg(m):
    """OdometryMsg -> (pose, bef) as the receiving handlers read it"""
    p, b = Pose6(), Pose6()
    _check(lib().loam_pose_from_msg(ctypes.byref(m), ctypes.byref(p), ctypes.byref(b)))
    return p.arr(), b.arr()
