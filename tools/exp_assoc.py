"""Diagnostic: cycle breakdown of the odometry association (build exp/libloam_ASSOCPH.so with -DLOAM_EXP_ASSOCPH)."""
import ctypes, importlib, os, sys
os.environ["LOAM_HIP_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "loam_velodyne-1_amd", "exp", "libloam_ASSOCPH.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
prevs, curs = sg.batch_problems(1024, base_seed=1000)
eng = loam.Engine(device=0)
eng.batch_upload(prevs, curs)
eng.batch_run(); eng.sync()
L = loam.lib()
arr = (ctypes.c_ulonglong * 8)()
L.loam_debug_assoc(arr)
a = list(arr)
eng.batch_run(); eng.sync()
L.loam_debug_assoc(arr)
d = [x - y for x, y in zip(arr, a)]
names = ["corner NN", "corner windows", "surf NN", "surf windows", "NN fallbacks (count)", "-", "-", "-"]
tot = sum(d[:4])
for n, v in zip(names, d):
    print(f"{n:22s} {v:14d} {100.0 * v / max(tot, 1):6.1f}%")
