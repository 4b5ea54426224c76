"""Diagnostic (GPU box): per-frame engine-vs-oracle mapping differences on the IMU stream."""
import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
import oracle_ctypes as oc
t0 = 0.0
sweeps = sg.stream_sweeps(24, 1, t0=t0)
imus = sg.imu_stream(t0 - 0.5, t0 + 2.5, seed=1)
cfg = dict(system_delay=2)
impls = [loam.Engine(loam.default_config(**cfg)), oc.Oracle(oc.default_config(**cfg))]
keys = ("mp_iters", "mp_rows_sum", "mp_stack", "mp_map_points", "mp_map_valid_points")
j = [0, 0]
frame = 0
for k, sw in enumerate(sweeps):
    outs = []
    for n, impl in enumerate(impls):
        while j[n] < len(imus) and imus[j[n]][0] <= t0 + 0.1 * (k + 1):
            impl.imu(*imus[j[n]]); j[n] += 1
        rc, f = impl.scan_registration(sw, stamp=t0 + 0.1 * k)
        if rc:
            outs.append(None); continue
        pub, pose, cl, sl, full = impl.odometry(f, stamp=t0 + 0.1 * k)
        if pub == 7:
            aft, bef, reg = impl.mapping(pose, cl, sl, full, stamp=t0 + 0.1 * k)
            st = impl.stats()
            outs.append((aft, reg, {q: st[q] for q in keys}, cl, sl))
        else:
            outs.append(None)
    if outs[0] is None:
        continue
    (a0, r0, s0, c0, l0), (a1, r1, s1, c1, l1) = outs
    print(frame, "aft", float(np.abs(a0 - a1).max()), "reg", r0.shape, r1.shape,
          float(np.abs(r0 - r1).max()) if r0.shape == r1.shape else -1, "in", float(np.abs(c0-c1).max()), float(np.abs(l0-l1).max()))
    print("   eng", s0); print("   ora", s1)
    frame += 1
