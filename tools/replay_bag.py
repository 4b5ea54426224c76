"""Replay a recorded rosbag v2.0 (e.g. the reference's nsh_indoor_outdoor.bag, when a local copy
exists) through the engine's node path — BASELINE configs 1-3 on recorded sweeps — and optionally
through the CPU oracle on the same messages.  Prints one JSON line: sweeps, scans/s, the final
odometry / mapping poses and (with --oracle) the largest pose difference.

    python tools/replay_bag.py BAG [--cloud-topic /velodyne_points] [--imu-topic /imu/data]
                               [--max-sweeps N] [--oracle] [--trajectory out.csv]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bag")
    ap.add_argument("--cloud-topic", default="/velodyne_points")
    ap.add_argument("--imu-topic", default="/imu/data")
    ap.add_argument("--max-sweeps", type=int, default=0)
    ap.add_argument("--oracle", action="store_true", help="also run the CPU oracle (test infrastructure)")
    ap.add_argument("--trajectory", default="", help="write stamp + mapping pose per published frame (CSV)")
    args = ap.parse_args()
    loam = importlib.import_module("loam_velodyne-1_amd")
    rb = importlib.import_module("loam_velodyne-1_amd.rosbag")
    t0 = time.perf_counter()
    out = rb.replay(args.bag, loam.Engine(loam.default_config()), args.cloud_topic, args.imu_topic,
                    args.max_sweeps or None)
    dt = time.perf_counter() - t0
    res = {"bag": args.bag, "sweeps": out["sweeps"], "seconds": dt, "scans_per_s": out["sweeps"] / dt if dt else None,
           "odometry_frames": len(out["odometry"]), "mapping_frames": len(out["mapping"]),
           "final_odometry": out["odometry"][-1][1].tolist() if out["odometry"] else None,
           "final_mapping": out["mapping"][-1][1].tolist() if out["mapping"] else None}
    if args.oracle:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as oc
        t0 = time.perf_counter()
        ref = rb.replay(args.bag, oc.Oracle(oc.default_config()), args.cloud_topic, args.imu_topic,
                        args.max_sweeps or None)
        res["oracle_seconds"] = time.perf_counter() - t0
        k = min(len(ref["mapping"]), len(out["mapping"]))
        if k:
            a = np.array([p for _, p in out["mapping"][:k]])
            b = np.array([p for _, p in ref["mapping"][:k]])
            res["max_abs_err_mapping"] = float(np.abs(a - b).max())
    if args.trajectory:
        with open(args.trajectory, "w") as f:
            f.write("stamp,rx,ry,rz,tx,ty,tz\n")
            for s, p in out["mapping"]:
                f.write(f"{s:.9f}," + ",".join(f"{v:.9g}" for v in p) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
