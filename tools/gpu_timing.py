import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
prevs, curs = sg.batch_problems(B)
e = loam.Engine(); e.batch_upload(prevs, curs)
e.batch_run(); e.sync()
for k in range(3):
    t0 = time.perf_counter(); e.batch_run(); t1 = time.perf_counter(); e.sync(); t2 = time.perf_counter()
    print(f"enqueue {1e3*(t1-t0):.2f} ms, sync {1e3*(t2-t1):.2f} ms")
