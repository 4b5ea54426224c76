"""Config 3 through loam_chain_sweep only (the device-resident node chain, bench.py
single_stream.device_chain): N sweeps of seed 1, one context, ms per processed sweep.  For kernel
traces of the streaming chain (rocprofv3 -- python3 tools/chain_bench.py [N]); diagnostic."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 220
    # further arguments: key=value launch choices (loam_set_tuning)
    tune = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[2:]}
    sweeps = sg.stream_sweeps(n, 1)
    warm = loam.Engine(loam.default_config(system_delay=1))
    warm.set_tuning(**tune)
    for k, s in enumerate(sweeps[:6]):
        warm.chain_sweep(s, stamp=0.1 * k)
    e = loam.Engine(loam.default_config())
    e.set_tuning(**tune)
    done, t = 0, 0.0
    for k, s in enumerate(sweeps):
        a = time.perf_counter()
        rc = e.chain_sweep(s, stamp=0.1 * k)[0]
        t += time.perf_counter() - a
        done += rc == 0
    print(f"chain {tune}: {done} sweeps processed, {1e3 * t / max(done, 1):.4f} ms per sweep")


if __name__ == "__main__":
    main()
