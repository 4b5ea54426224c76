"""diagnostic: throughput of the batch split over K engine contexts (one HIP stream each) that run
concurrently on one GPU, against one context holding the whole batch"""
import importlib, sys, time
sys.path.insert(0, '/root/repo')
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
B = 1024
prevs, curs = sg.batch_problems(B, base_seed=1000)
for K in (1, 2, 4):
    engs = []
    per = B // K
    for k in range(K):
        e = loam.Engine(device=0)
        e.batch_upload(prevs[k * per:(k + 1) * per], curs[k * per:(k + 1) * per])
        engs.append(e)
    def step():
        for e in engs:
            e.batch_run()
        for e in engs:
            e.sync()
    for _ in range(3):
        step()
    t = time.perf_counter()
    for _ in range(10):
        step()
    dt = (time.perf_counter() - t) / 10
    print(f"K={K}: {dt*1e3:.2f} ms/step, {B/dt:.0f} problems/s", flush=True)
    del engs
