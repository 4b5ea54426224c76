"""How long the host takes to enqueue one pipelined batch step (loam_batch_run without a sync)
against the device's step time, at the 8-GPU share (128 problems) or another batch size.  If the
enqueue time per step approaches the step time, the host, not the GPU, paces the pipeline.
Diagnostic.   python tools/host_enqueue.py [P] [steps] [key=value ...]"""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    tune = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[3:]}
    prevs, curs = sg.batch_problems(P, base_seed=1000)
    e = loam.Engine()
    e.set_tuning(**tune)
    e.batch_upload(prevs, curs)
    for _ in range(3):
        e.batch_run()
    e.sync()
    enq = []
    a = time.perf_counter()
    for _ in range(K):
        b = time.perf_counter()
        e.batch_run()
        enq.append(time.perf_counter() - b)
    c = time.perf_counter()
    e.sync()
    d = time.perf_counter()
    enq.sort()
    print(f"P={P} {tune}: step {1e3 * (d - a) / K:.3f} ms (enqueue loop {1e3 * (c - a) / K:.3f} ms/step, "
          f"median call {1e3 * enq[K // 2]:.3f} ms, max {1e3 * enq[-1]:.3f} ms)")
    e.close()


if __name__ == "__main__":
    main()
