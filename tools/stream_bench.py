"""Configs 3 and 5 timing (not the bench.py metric): the streaming node path one sweep at a time
(loam_scan_registration -> loam_odometry -> loam_mapping on every 2nd sweep, host buffers in and
out per call, as the ROS nodes would call it) on one GPU, next to the CPU oracle on the same
sweeps; and the single HDL-64E problem (config 5).  Prints one JSON line."""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
import oracle_ctypes as oc  # noqa: E402


def stream(impl, sweeps):
    poses, t_sr, t_od, t_mp, n = [], 0.0, 0.0, 0.0, 0
    for k, sw in enumerate(sweeps):
        a = time.perf_counter()
        rc, f = impl.scan_registration(sw, stamp=0.1 * k)
        b = time.perf_counter()
        t_sr += b - a
        if rc != 0:
            continue
        n += 1
        pub, pose, cl, sl, full = impl.odometry(f, stamp=0.1 * k)
        c = time.perf_counter()
        t_od += c - b
        if pub == 7:
            aft, bef, reg = impl.mapping(pose, cl, sl, full)
            poses.append(aft)
        t_mp += time.perf_counter() - c
    return np.array(poses), n, t_sr, t_od, t_mp


def main():
    n_sweeps = int(os.environ.get("STREAM_SWEEPS", "220"))
    n_cpu = int(os.environ.get("STREAM_CPU_SWEEPS", "80"))
    sweeps = sg.stream_sweeps(n_sweeps, 1)
    eng = loam.Engine(loam.default_config())
    stream(loam.Engine(loam.default_config(system_delay=1)), sweeps[:6])  # warm-up (allocations, code load)
    pg, ng, a, b, c = stream(eng, sweeps)
    gpu = {"sweeps_processed": ng, "scans_per_s": ng / (a + b + c), "ms_sr": 1e3 * a / ng, "ms_od": 1e3 * b / ng,
           "ms_mp_per_processed": 1e3 * c / ng}
    po, no, a2, b2, c2 = stream(oc.Oracle(oc.default_config()), sweeps[:n_cpu])
    cpu = {"sweeps_processed": no, "scans_per_s": no / (a2 + b2 + c2), "cores": 1}
    k = min(len(po), len(pg))
    err = float(np.abs(pg[:k] - po[:k]).max()) if k else None
    # config 5: one HDL-64E problem through the batch path (batch of one) and the oracle
    prev, cur = sg.single_problem(2, lidar=sg.HDL64)
    cfg = loam.default_config(n_rings=64, ring_model=loam.RING_LINEAR, max_points=160000, od_max_iter=100,
                              mp_max_iter=20)
    e5 = loam.Engine(cfg)
    e5.batch_upload([prev], [cur])
    e5.batch_run(); e5.sync()
    reps = 5
    t = time.perf_counter()
    for _ in range(reps):
        e5.batch_run()
    e5.sync()
    g5 = (time.perf_counter() - t) / reps
    od5, aft5, _ = e5.batch_download()
    t = time.perf_counter()
    od5o, aft5o, _ = oc.problem(prev, cur, oc.default_config(n_rings=64, ring_model=1, max_points=160000,
                                                             od_max_iter=100, mp_max_iter=20))
    c5 = time.perf_counter() - t
    out = {"config3_stream": {"gpu": gpu, "cpu_oracle": cpu, "mapping_poses_compared": k, "max_abs_err": err},
           "config5_hdl64_problem": {"gpu_ms": 1e3 * g5, "cpu_ms": 1e3 * c5,
                                     "max_abs_err": float(max(np.abs(od5[0] - od5o).max(), np.abs(aft5[0] - aft5o).max()))}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
