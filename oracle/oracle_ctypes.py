"""ctypes binding of liboracle.so — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).

The oracle is the CPU restatement of the reference hot path (oracle/oracle.cpp); PARITY UNPINNED
(the reference has no tests or fixtures and cannot be built here)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


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


class Config(ctypes.Structure):
    _fields_ = [("n_rings", ctypes.c_uint32), ("ring_model", ctypes.c_uint32),
                ("ring_lo_deg", ctypes.c_float), ("ring_hi_deg", ctypes.c_float),
                ("system_delay", ctypes.c_uint32), ("max_points", ctypes.c_uint32),
                ("od_max_iter", ctypes.c_uint32), ("mp_max_iter", ctypes.c_uint32),
                ("skip_frame_num", ctypes.c_uint32), ("map_capacity", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "n_raw", "n_ring", "n_sharp", "n_less_sharp", "n_flat", "n_less_flat",
        "od_iters", "od_assoc_rounds", "od_rows_sum", "od_corner_last", "od_surf_last", "od_queries",
        "od_assoc_points",
        "mp_iters", "mp_rows_sum", "mp_stack", "mp_map_points", "mp_map_valid_points", "mp_stack_iters",
        "mp_fits", "od_query_iters", "od_row_evals",
        "bytes_sr", "bytes_od", "bytes_mp")] + [(n, ctypes.c_double) for n in ("ms_sr", "ms_od", "ms_mp")] + \
        [(n, ctypes.c_uint64) for n in ("od_degenerate_steps", "od_nan_skips", "mp_degenerate_steps",
                                        "mp_grid_shifts",
                                        # engine-only search counters (zero here: the oracle's kd-tree
                                        # does different work)
                                        "mp_nn_candidates", "mp_nn_cells", "od_assoc_gathered",
                                        "od_assoc_boxes")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


def lib():
    global _LIB
    if _LIB is None:
        # LOAM_ORACLE_LIB: the sanitizer build (make -C oracle asan -> liboracle_asan.so)
        path = os.environ.get("LOAM_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so not built (make -C oracle)")
        L = ctypes.CDLL(path)
        L.oracle_create.restype = ctypes.c_void_p
        L.oracle_create.argtypes = [ctypes.POINTER(Config)]
        L.oracle_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_config_default.argtypes = [ctypes.POINTER(Config)]
        L.oracle_scan_registration.argtypes = [ctypes.c_void_p, ctypes.c_double, CloudIn,
                                               ctypes.POINTER(Features)]
        L.oracle_odometry.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.POINTER(Features),
                                      ctypes.POINTER(Pose6), ctypes.POINTER(CloudOut),
                                      ctypes.POINTER(CloudOut), ctypes.POINTER(CloudOut),
                                      ctypes.POINTER(ctypes.c_int)]
        L.oracle_mapping.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.POINTER(Pose6),
                                     ctypes.POINTER(CloudOut), ctypes.POINTER(CloudOut),
                                     ctypes.POINTER(CloudOut), ctypes.POINTER(Pose6),
                                     ctypes.POINTER(Pose6), ctypes.POINTER(CloudOut)]
        L.oracle_mapping_surround.argtypes = [ctypes.c_void_p, ctypes.POINTER(CloudOut),
                                              ctypes.POINTER(ctypes.c_int)]
        L.oracle_maintenance.argtypes = [ctypes.POINTER(Pose6)] * 4
        L.oracle_imu.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_double)]
        L.oracle_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(Stats)]
        L.oracle_problem.argtypes = [ctypes.POINTER(Config), CloudIn, CloudIn, ctypes.POINTER(Pose6),
                                     ctypes.POINTER(Pose6), ctypes.POINTER(Stats)]
        L.oracle_problem_with_od.argtypes = [ctypes.POINTER(Config), CloudIn, CloudIn, ctypes.POINTER(Pose6),
                                             ctypes.POINTER(Pose6), ctypes.POINTER(Pose6), ctypes.POINTER(Stats)]
        L.oracle_voxel_grid.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                        ctypes.c_void_p, ctypes.c_int]
        L.oracle_knn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_qr_solve.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p]
        L.oracle_jacobi.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_lu_inv.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.oracle_pose_through_msg.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_msg_orientation.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _LIB = L
    return _LIB


def default_config(**kw):
    c = Config()
    lib().oracle_config_default(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def cloud_in(a):
    a = np.ascontiguousarray(a, np.float32)
    return CloudIn(a.ctypes.data, a.shape[0], a.shape[1] * 4), a


class OutBuf:
    """caller-owned output cloud storage"""

    def __init__(self, cap):
        self.arr = np.zeros((max(cap, 1), 4), np.float32)
        self.c = CloudOut(self.arr.ctypes.data, 0, cap)

    def get(self):
        return self.arr[:self.c.count].copy()


def make_features(cap):
    bufs = [OutBuf(cap) for _ in range(5)]
    f = Features(*[b.c for b in bufs])
    return f, bufs


def features_to_dict(f, bufs):
    # ctypes copies the CloudOut structs into Features: read counts from f
    names = ["full", "sharp", "less_sharp", "flat", "less_flat"]
    d = {n: b.arr[:getattr(f, n).count].copy() for n, b in zip(names, bufs)}
    d["imu_trans"] = np.array(f.imu_trans[:], np.float32)
    return d


class Oracle:
    """stateful streaming oracle: one object = the four reference nodes"""

    def __init__(self, cfg=None, cap=200000):
        self.cfg = cfg or default_config()
        self.h = lib().oracle_create(ctypes.byref(self.cfg))
        self.cap = cap

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_destroy(self.h)
            self.h = None

    def imu(self, stamp, quat_xyzw, lin_acc):
        q = (ctypes.c_double * 4)(*[float(v) for v in quat_xyzw])
        a = (ctypes.c_double * 3)(*[float(v) for v in lin_acc])
        assert lib().oracle_imu(self.h, stamp, q, a) == 0

    def scan_registration(self, raw, stamp=0.0):
        ci, keep = cloud_in(raw)
        f, bufs = make_features(self.cap)
        rc = lib().oracle_scan_registration(self.h, stamp, ci, ctypes.byref(f))
        if rc != 0:
            return rc, None
        return 0, features_to_dict(f, bufs)

    def odometry(self, feats, stamp=0.0):
        keep = []
        cl = []
        for n in ["full", "sharp", "less_sharp", "flat", "less_flat"]:
            a = np.ascontiguousarray(feats[n], np.float32).reshape(-1, 4)
            keep.append(a)
            cl.append(CloudOut(a.ctypes.data if a.shape[0] else None, a.shape[0], a.shape[0]))
        f = Features(*cl)
        if "imu_trans" in feats:
            f.imu_trans[:] = [float(v) for v in feats["imu_trans"]]
        pose = Pose6()
        outs = [OutBuf(self.cap) for _ in range(3)]
        pub = ctypes.c_int(0)
        rc = lib().oracle_odometry(self.h, stamp, ctypes.byref(f), ctypes.byref(pose),
                                   ctypes.byref(outs[0].c), ctypes.byref(outs[1].c),
                                   ctypes.byref(outs[2].c), ctypes.byref(pub))
        assert rc == 0, rc
        return pub.value, pose.arr(), outs[0].get(), outs[1].get(), outs[2].get()

    def mapping(self, odom_sum, corner, surf, full, stamp=0.0):
        keep = []
        cl = []
        for a in (corner, surf, full):
            a = np.ascontiguousarray(a, np.float32).reshape(-1, 4)
            keep.append(a)
            cl.append(CloudOut(a.ctypes.data if a.shape[0] else None, a.shape[0], a.shape[0]))
        aft, bef = Pose6(), Pose6()
        reg = OutBuf(max(full.shape[0], 1))
        rc = lib().oracle_mapping(self.h, stamp, ctypes.byref(Pose6.of(odom_sum)), ctypes.byref(cl[0]),
                                  ctypes.byref(cl[1]), ctypes.byref(cl[2]), ctypes.byref(aft),
                                  ctypes.byref(bef), ctypes.byref(reg.c))
        assert rc == 0, rc
        return aft.arr(), bef.arr(), reg.get()

    def mapping_surround(self):
        """/laser_cloud_surround of the last mapping frame, or None when it is not published"""
        pub = ctypes.c_int(0)
        out = OutBuf(1)
        rc = lib().oracle_mapping_surround(self.h, ctypes.byref(out.c), ctypes.byref(pub))
        if rc == -2:
            out = OutBuf(int(out.c.count))
            rc = lib().oracle_mapping_surround(self.h, ctypes.byref(out.c), ctypes.byref(pub))
        assert rc == 0, rc
        return out.get() if pub.value else None

    def stats(self):
        s = Stats()
        lib().oracle_get_stats(self.h, ctypes.byref(s))
        return s.as_dict()


def maintenance(odom_sum, bef, aft):
    out = Pose6()
    lib().oracle_maintenance(ctypes.byref(Pose6.of(odom_sum)), ctypes.byref(Pose6.of(bef)),
                             ctypes.byref(Pose6.of(aft)), ctypes.byref(out))
    return out.arr()


def problem(prev, cur, cfg=None):
    """one config-4 problem: returns (odometry transformSum, mapped Aft pose, stats dict)"""
    cfg = cfg or default_config()
    a, ka = cloud_in(prev)
    b, kb = cloud_in(cur)
    od, aft, st = Pose6(), Pose6(), Stats()
    rc = lib().oracle_problem(ctypes.byref(cfg), a, b, ctypes.byref(od), ctypes.byref(aft),
                              ctypes.byref(st))
    assert rc == 0, rc
    return od.arr(), aft.arr(), st.as_dict()


def problem_with_od(prev, cur, od_transform, cfg=None):
    """problem() with the odometry's L-M solution replaced by od_transform (6 floats) before its
    accumulation and TransformToEnd: the reference's mapping for that odometry result"""
    cfg = cfg or default_config()
    a, ka = cloud_in(prev)
    b, kb = cloud_in(cur)
    od, aft, st = Pose6(), Pose6(), Stats()
    rc = lib().oracle_problem_with_od(ctypes.byref(cfg), a, b, ctypes.byref(Pose6.of(od_transform)),
                                      ctypes.byref(od), ctypes.byref(aft), ctypes.byref(st))
    assert rc == 0, rc
    return od.arr(), aft.arr(), st.as_dict()
