"""Streaming A/B of engine builds (config 3 sequential, seed 1, 220 sweeps): per library (argv), in a
child process with LOAM_HIP_LIB set, the per-sweep time of the three node calls (best of 3 runs)
and per node.  python tools/exp_stream.py lib1.so lib2.so ...   (GPU)"""
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")

CHILD = r'''
import importlib, json, sys, time
import numpy as np
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
sweeps = sg.stream_sweeps(220, 1)
best = None
for rep in range(3):
    e = loam.Engine(loam.default_config())
    t = [0.0, 0.0, 0.0]; n = 0; poses = []
    for k, s in enumerate(sweeps):
        a = time.perf_counter()
        rc, f = e.scan_registration(s, stamp=0.1 * k)
        b = time.perf_counter(); t[0] += b - a
        if rc:
            continue
        n += 1
        pub, pose, cl, sl, full = e.odometry(f, stamp=0.1 * k)
        c = time.perf_counter(); t[1] += c - b
        if pub == 7:
            poses.append(e.mapping(pose, cl, sl, full, stamp=0.1 * k)[0])
        t[2] += time.perf_counter() - c
    e.close()
    tot = sum(t) / n * 1e3
    if best is None or tot < best["ms_per_sweep"]:
        best = {"ms_per_sweep": tot, "sr": t[0] / n * 1e3, "od": t[1] / n * 1e3, "mp": t[2] / n * 1e3,
                "last": np.array(poses[-1]).tolist()}
print(json.dumps(best))
'''

for lib in sys.argv[1:]:
    env = dict(os.environ, LOAM_HIP_LIB=os.path.abspath(lib))
    r = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env, capture_output=True,
                       text=True, timeout=300)
    if r.returncode:
        print(lib, "FAILED", r.stderr[-2000:])
        sys.exit(1)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    print(os.path.basename(lib), json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items()}),
          flush=True)
