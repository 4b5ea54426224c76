"""Experiment: does one GPU finish a batch of P problems sooner as K concurrent sub-batches (K
engine contexts, each with its own streams) than as one?  Prints ms per batch for each split.
    python tools/exp_lanes.py [P] [K ...]      (GPU)"""
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")

P = int(sys.argv[1]) if len(sys.argv) > 1 else 128
splits = [int(k) for k in sys.argv[2:]] or [1, 2, 4]
prevs, curs = sg.batch_problems(P, base_seed=1000)
ref = None
for K in splits:
    engs = []
    for k in range(K):
        e = loam.Engine()
        e.batch_upload(prevs[k * P // K:(k + 1) * P // K], curs[k * P // K:(k + 1) * P // K])
        engs.append(e)
    for _ in range(3):
        for e in engs:
            e.batch_run()
        for e in engs:
            e.sync()
    best = 1e9
    for rep in range(5):
        t0 = time.perf_counter()
        for _ in range(10):
            for e in engs:
                e.batch_run()
            for e in engs:
                e.sync()
        best = min(best, (time.perf_counter() - t0) / 10 * 1e3)
    aft = np.concatenate([e.batch_download()[1] for e in engs])
    if ref is None:
        ref = aft
    same = bool(np.array_equal(aft, ref))
    print(f"P={P} K={K}: {best:.3f} ms/batch  {P / best * 1e3:.0f} problems/s  same_poses={same}", flush=True)
    for e in engs:
        e.close()
