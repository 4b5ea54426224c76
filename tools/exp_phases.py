"""Diagnostic: cycle breakdown of k_sr_select phases (build exp/libloam_PHASES.so with -DLOAM_EXP_PHASES)."""
import ctypes, importlib, os, sys
os.environ["LOAM_HIP_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "loam_velodyne-1_amd", "exp", "libloam_PHASES.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
prevs, curs = sg.batch_problems(1024, base_seed=1000)
eng = loam.Engine(device=0)
eng.batch_upload(prevs, curs)
eng.batch_run(); eng.sync()
L = loam.lib()
arr = (ctypes.c_ulonglong * 8)()
L.loam_debug_phases(arr)
a = list(arr)
eng.batch_run(); eng.sync()
L.loam_debug_phases(arr)
d = [x - y for x, y in zip(arr, a)]
tot = sum(d)
names = ["pick: load+compact", "pick: sort", "pick: sharp walk", "pick: flat walk", "pick: candidates", "pick: setup route", "pick: setup pk window", "-"] if "--pick" in sys.argv else ["load+keys", "ring sort", "greedy+cand", "seq wb + vg bbox", "vg keys", "vg sort", "vg heads", "-"]
for n, v in zip(names, d):
    print(f"{n:18s} {v:14d} {100.0 * v / max(tot, 1):6.1f}%")
