"""Synthetic sweep scenarios for the BASELINE.json configs (test / bench input only).

The recorded bags the reference is validated on (nsh_indoor_outdoor.bag etc., /root/reference/
README.md:22-35) are not available offline, so every config runs on seeded synthetic sweeps from
libloam_synth.so (see synth/synth.cpp for the sensor model).  SURVEY.md §8(d) fixes the shapes:

  config 1/2  one VLP-16 problem (prev sweep, cur sweep), indoor scene, seed 0
  config 3    220 VLP-16 sweeps at 10 Hz along a loop, seed 1
  config 4    1024 independent problems, random planes + edges scenes, seeds 1000..2023
  config 5    one HDL-64E problem, indoor scene, seed 2
"""
import ctypes
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

SCENE_INDOOR, SCENE_RANDOM = 0, 1
VLP16, HDL64 = 0, 1
SCAN_PERIOD = 0.1
START_AZ = math.pi          # velodyne-frame azimuth of the first firing of every sweep
SIGMA = 0.01                # range noise (m)


def lib():
    global _LIB
    if _LIB is None:
        path = os.environ.get("LOAM_SYNTH_LIB") or os.path.join(_HERE, "synth", "libloam_synth.so")
        if not os.path.exists(path):
            raise RuntimeError("libloam_synth.so not built (run __graft_entry__.build())")
        L = ctypes.CDLL(path)
        L.synth_scene_create.restype = ctypes.c_void_p
        L.synth_scene_create.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.synth_scene_destroy.argtypes = [ctypes.c_void_p]
        L.synth_max_points.argtypes = [ctypes.c_int]
        L.synth_sweep.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_uint64, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_void_p, ctypes.c_int]
        L.synth_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                                  ctypes.c_double, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_int]
        _LIB = L
    return _LIB


class Scene:
    def __init__(self, kind, seed):
        self.h = lib().synth_scene_create(kind, seed)

    def __del__(self):
        if getattr(self, "h", None) and _LIB is not None:
            _LIB.synth_scene_destroy(self.h)
            self.h = None


def sweep(scene, lidar, pose0, pose1, noise_seed, sigma=SIGMA):
    """One sweep as an (n, 4) float32 array (x, y, z, laser) in firing order."""
    cap = lib().synth_max_points(lidar)
    out = np.zeros((cap, 4), np.float32)
    p0 = np.ascontiguousarray(pose0, np.float64)
    p1 = np.ascontiguousarray(pose1, np.float64)
    n = lib().synth_sweep(scene.h, lidar, p0.ctypes.data, p1.ctypes.data, noise_seed, sigma,
                          START_AZ, out.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("synth_sweep overflow")
    return out[:n].copy()


def sweeps_batch(scenes, lidar, poses0, poses1, seeds, sigma=SIGMA, nthreads=None):
    """Many sweeps in parallel: returns (list of (n_i,4) arrays)."""
    n = len(scenes)
    cap = lib().synth_max_points(lidar)
    out = np.zeros((n, cap, 4), np.float32)
    counts = np.zeros(n, np.int32)
    handles = (ctypes.c_void_p * n)(*[s.h for s in scenes])
    p0 = np.ascontiguousarray(poses0, np.float64)
    p1 = np.ascontiguousarray(poses1, np.float64)
    sd = np.ascontiguousarray(seeds, np.uint64)
    nt = nthreads or min(16, os.cpu_count() or 1)
    rc = lib().synth_batch(n, handles, lidar, p0.ctypes.data, p1.ctypes.data, sd.ctypes.data,
                           sigma, START_AZ, out.ctypes.data, cap, counts.ctypes.data, nt)
    if rc != 0:
        raise RuntimeError("synth_batch overflow")
    return [out[i, :counts[i]] for i in range(n)]


def loop_pose(t, radius=6.0, speed=1.0, theta0=-math.pi / 2):
    """Indoor loop: circle of `radius` m at `speed` m/s (yaw rate = speed/radius ~ 9.5 deg/s)."""
    th = theta0 + speed / radius * t
    return np.array([radius * math.cos(th), radius * math.sin(th), 0.0,
                     0.0, 0.0, th + math.pi / 2])


def stream_sweeps(n_sweeps, seed, lidar=VLP16, t0=0.0):
    """Config 3 (and the 2-sweep problems of configs 1/2/5): consecutive sweeps on the loop."""
    scene = Scene(SCENE_INDOOR, seed)
    p0 = [loop_pose(t0 + k * SCAN_PERIOD) for k in range(n_sweeps)]
    p1 = [loop_pose(t0 + (k + 1) * SCAN_PERIOD) for k in range(n_sweeps)]
    seeds = [seed * 1000003 + k for k in range(n_sweeps)]
    return sweeps_batch([scene] * n_sweeps, lidar, p0, p1, seeds)


def single_problem(seed=0, lidar=VLP16):
    """Configs 1/2 (VLP-16, seed 0) and 5 (HDL-64E, seed 2): (prev, cur) sweeps."""
    prev, cur = stream_sweeps(2, seed, lidar=lidar, t0=1.0)
    return prev, cur


def batch_problems(n, base_seed=1000, lidar=VLP16, nthreads=None):
    """Config 4: n independent problems; problem i uses seed base_seed+i, its own random
    planes+edges scene and random constant motion |t| <= 0.3 m, |r| <= 3 deg per sweep.
    Returns (prev_list, cur_list)."""
    scenes, p0s, p1s, seeds = [], [], [], []
    for i in range(n):
        s = base_seed + i
        rng = np.random.default_rng(s)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        trans = d * rng.uniform(0.0, 0.3)
        trans[2] *= 0.3
        rot = rng.uniform(-1.0, 1.0, size=3)
        rot *= math.radians(rng.uniform(0.0, 3.0)) / max(np.linalg.norm(rot), 1e-9)
        start = np.concatenate([rng.uniform(-1, 1, size=3) * [1.0, 1.0, 0.2],
                                rng.uniform(-1, 1, size=3) * [0.02, 0.02, math.pi]])
        inc = np.concatenate([trans, rot])
        sc = Scene(SCENE_RANDOM, s)
        scenes += [sc, sc]
        p0s += [start, start + inc]
        p1s += [start + inc, start + 2 * inc]
        seeds += [s * 2 + 1, s * 2 + 2]
    sw = sweeps_batch(scenes, lidar, p0s, p1s, seeds, nthreads=nthreads)
    return sw[0::2], sw[1::2]


def quat_from_rpy(roll, pitch, yaw):
    """tf::Quaternion::setRPY as (x, y, z, w)"""
    hy, hp, hr = yaw * 0.5, pitch * 0.5, roll * 0.5
    cy, sy, cp, sp, cr, sr = math.cos(hy), math.sin(hy), math.cos(hp), math.sin(hp), math.cos(hr), math.sin(hr)
    return (sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
            cr * cp * cy + sr * sp * sy)


def imu_stream(t_begin, t_end, rate=100.0, seed=0, radius=6.0, speed=1.0, tilt_deg=0.3):
    """/imu/data messages (stamp, quat_xyzw, linear_acceleration) for the config-3 loop: the
    vehicle yaw of loop_pose, a small seeded roll / pitch wobble, and the specific force of the
    circular motion (centripetal acceleration to the left, gravity up) in the IMU frame (x forward,
    y left, z up).  Deterministic; stamps strictly increasing."""
    rng = np.random.default_rng(seed)
    ph = rng.uniform(0, 2 * math.pi, size=2)
    out = []
    n = int(round((t_end - t_begin) * rate))
    for k in range(n + 1):
        t = t_begin + k / rate
        yaw = loop_pose(t, radius, speed)[5]
        roll = math.radians(tilt_deg) * math.sin(1.3 * t + ph[0])
        pitch = math.radians(tilt_deg) * math.sin(0.9 * t + ph[1])
        acc = (0.0, speed * speed / radius, 9.81)
        out.append((t, quat_from_rpy(roll, pitch, yaw), acc))
    return out
