"""Config-3 chain (loam_chain_sweep) per-sweep wall time against the GPU spans the engine records
(loam_stats ms_sr / ms_od / ms_mp, HIP events around each node's kernels): what is host work,
copies and synchronisation.  Diagnostic; run on the GPU box from the repo root."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")

sweeps = sg.stream_sweeps(220, 1)
e = loam.Engine(loam.default_config())
tot = {"wall": 0.0, "sr": 0.0, "od": 0.0, "mp": 0.0, "n": 0, "nmap": 0}
for k, s in enumerate(sweeps):
    a = time.perf_counter()
    rc, pub, od, aft, bef, _ = e.chain_sweep(s, stamp=0.1 * k)
    w = time.perf_counter() - a
    if rc or k < 30:
        continue
    st = e.stats()
    tot["wall"] += w * 1e3
    tot["sr"] += st["ms_sr"]
    tot["od"] += st["ms_od"]
    tot["mp"] += st["ms_mp"] if aft is not None else 0.0
    tot["n"] += 1
    tot["nmap"] += aft is not None
n = tot["n"]
print(f"sweeps {n} (mapping on {tot['nmap']}): wall {tot['wall'] / n:.4f} ms, sr {tot['sr'] / n:.4f}, "
      f"od {tot['od'] / n:.4f}, mp {tot['mp'] / n:.4f}, rest {(tot['wall'] - tot['sr'] - tot['od'] - tot['mp']) / n:.4f}")
