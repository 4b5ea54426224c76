"""Benchmark: scans/sec of the LOAM hot path (scan registration + odometry L-M + mapping L-M) on
MI355X, BASELINE.json config 4 shape: independent synthetic VLP-16 problems, sharded across ranks.

One step = one pass of the whole hot path over this rank's batch of problems, inputs resident in
HBM: scan registration of both sweeps of every problem, odometry seeded from prev and solved on
cur, mapping of prev into an empty map and solved for cur.  Weak scaling: every
rank owns --batch problems (seeds 1000 + global index); the data path has no collective; one RCCL
all-gather of the poses after the timed steps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--cpu-seconds S]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "scans/sec (odometry+mapping L-M solve) VLP-16 sweep, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def kernel_bytes(st):
    """Algorithmic HBM bytes of each kernel over one step of the whole batch (SURVEY.md §8(d),
    split by the kernel that moves them)."""
    feats = 16 * (st["n_sharp"] + st["n_less_sharp"] + st["n_flat"] + st["n_less_flat"])
    return {
        "k_sr_ring_sort": 16 * st["n_raw"] + 16 * st["n_ring"],
        "k_sr_features": 16 * st["n_ring"],
        "k_sr_select": 16 * st["n_ring"] + feats,
        "k_od_solve": st["bytes_od"],
        # per iteration: every stored row's coefficient (16 B) + accept flag (1 B) read back (Q12:
        # all rows so far re-evaluated at the current transform), the query point read (16 B) and
        # its coefficient + flag written (17 B)
        "k_od_rows": 17 * st["od_row_evals"] + 33 * st["od_query_iters"],
        # per iteration: stack point 16 B (k_mp_nn), 5 neighbours 80 B read and the row (16 B point +
        # 16 B coeff) written (k_mp_fit)
        "k_mp_nn": 16 * st["mp_stack_iters"],
        "k_mp_fit": 80 * st["mp_stack_iters"] + 32 * st["mp_rows_sum"],
        # rows read back for JtJ
        "k_mp_iter": 32 * st["mp_rows_sum"],
    }


def stream_leg(loam, sg, n_sweeps, n_cpu):
    """Config 3 (streaming, seed 1): scan registration -> odometry -> mapping on every published
    frame, one sweep at a time on one GPU context, next to the CPU oracle on the first sweeps."""
    sweeps = sg.stream_sweeps(n_sweeps, 1)

    def run(impl, sw):
        poses, n, t = [], 0, 0.0
        for k, s in enumerate(sw):
            a = time.perf_counter()
            rc, f = impl.scan_registration(s, stamp=0.1 * k)
            if rc == 0:
                n += 1
                pub, pose, cl, sl, full = impl.odometry(f, stamp=0.1 * k)
                if pub == 7:
                    poses.append(impl.mapping(pose, cl, sl, full)[0])
            t += time.perf_counter() - a
        return np.array(poses), n, t

    warm = loam.Engine(loam.default_config(system_delay=1))
    run(warm, sweeps[:6])
    pg, ng, tg = run(loam.Engine(loam.default_config()), sweeps)
    out = {"config": "config3: VLP-16 stream (seed 1), systemDelay 20, mapping every 2nd frame",
           "sweeps_processed": ng, "scans_per_s": ng / tg, "ms_per_sweep": 1e3 * tg / max(ng, 1)}
    if n_cpu > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as oc
        po, no, tc = run(oc.Oracle(oc.default_config()), sweeps[:n_cpu])
        k = min(len(po), len(pg))
        out["cpu_oracle"] = {"sweeps_processed": no, "scans_per_s": no / tc, "cores": 1, "kind": "port"}
        out["speedup_vs_cpu"] = out["scans_per_s"] / out["cpu_oracle"]["scans_per_s"]
        out["max_abs_err_mapping"] = float(np.abs(pg[:k] - po[:k]).max()) if k else None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--stream-sweeps", type=int, default=120, help="config-3 streaming leg (0: skip)")
    ap.add_argument("--stream-cpu-sweeps", type=int, default=40)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
        dist = tdist

    loam = importlib.import_module("loam_velodyne-1_amd")
    sg = importlib.import_module("loam_velodyne-1_amd.synthgen")

    B = args.batch
    prevs, curs = sg.batch_problems(B, base_seed=1000 + rank * B)
    eng = loam.Engine(device=local)
    eng.batch_upload(prevs, curs)

    def sync():
        eng.sync()

    for _ in range(args.warmup):
        eng.batch_run()
    sync()

    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.batch_run()
    sync()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()

    od, aft, st = eng.batch_download()

    # host-buffer rate: the same batch handed over from host memory, upload + one step
    a = time.perf_counter()
    eng.batch_upload(prevs, curs)
    sync()
    upload_s = time.perf_counter() - a

    # per-kernel device times of the same workload (HIP events on the engine stream), untimed
    eng.set_profiling(True)
    for _ in range(args.profile_steps):
        eng.batch_run()
    eng.batch_download()
    ktimes = eng.kernel_times()
    eng.set_profiling(False)

    if dist:  # the one collective: gather every rank's poses (RCCL all-gather)
        import torch
        mine = torch.from_numpy(np.concatenate([od, aft], axis=1).astype(np.float32)).to(f"cuda:{local}")
        allp = torch.empty((world * B, 12), dtype=torch.float32, device=f"cuda:{local}")
        dist.all_gather_into_tensor(allp, mine)
        torch.cuda.synchronize()

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed

    # roofline of the dominant kernel: algorithmic bytes per launch / average launch duration
    kb = kernel_bytes(st)
    dom = max(ktimes.items(), key=lambda kv: kv[1][0])[0] if ktimes else None
    roof = None
    if dom:
        tot_ms, launches = ktimes[dom]
        avg_ms = tot_ms / max(launches, 1)
        nbytes = kb.get(dom)
        launches_per_step = launches / max(args.profile_steps, 1)
        per_launch = nbytes / launches_per_step if nbytes is not None else None
        achieved = per_launch / (avg_ms * 1e-3) / 1e9 if per_launch is not None else None
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tpath):
            try:
                traffic = json.load(open(tpath)).get(dom)
            except Exception:
                traffic = None
        roof = {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved is not None else None,
                "traffic": traffic, "avg_launch_ms": avg_ms, "algorithmic_bytes_per_launch": per_launch}

    # CPU baseline: the oracle (single-thread C++ restatement) on a bounded sample, N=1 only
    cpu = None
    parity = None
    if world == 1 and args.cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as oc
        n_done, t_cpu, err_od, err_mp = 0, 0.0, 0.0, 0.0
        while n_done < B and (t_cpu < args.cpu_seconds or n_done < 4):
            a = time.perf_counter()
            od_o, aft_o, _ = oc.problem(prevs[n_done], curs[n_done])
            t_cpu += time.perf_counter() - a
            err_od = max(err_od, float(np.abs(od[n_done] - od_o).max()))
            err_mp = max(err_mp, float(np.abs(aft[n_done] - aft_o).max()))
            n_done += 1
        model = "unknown CPU"
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        cpu = {"value": n_done / t_cpu, "unit": "scans/s", "cores": 1, "kind": "port",
               "sample": f"first {n_done} problems of the batch (seeds 1000..{999 + n_done}), "
                         f"oracle/liboracle.so -O3 single thread on {model} ({os.cpu_count()} logical CPUs "
                         f"visible), {t_cpu:.1f} s"}
        parity = {"problems_checked": n_done, "max_abs_err_odometry": err_od, "max_abs_err_mapping": err_mp}

    stage_ms = {k: round(v[0] / max(args.profile_steps, 1), 4) for k, v in sorted(ktimes.items())}
    # the same achieved-vs-peak figure for every kernel with an algorithmic byte count
    roof_all = {}
    for k, nbytes in kb.items():
        if k in ktimes and ktimes[k][0] > 0:
            gbs = nbytes / (ktimes[k][0] / max(args.profile_steps, 1) * 1e-3) / 1e9  # bytes per step / s per step
            roof_all[k] = {"achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                           "ms_per_step": round(ktimes[k][0] / max(args.profile_steps, 1), 4)}

    # single-stream latency path (BASELINE configs 2/3): one context fed sweep by sweep through the
    # node-level C-ABI with host buffers in and out, as the ROS nodes would call it (not the metric)
    stream = None
    if world == 1 and args.stream_sweeps > 0:
        stream = stream_leg(loam, sg, args.stream_sweeps, args.stream_cpu_sweeps)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32 (fp64 JtJ accumulation)",
        "data": "synthetic (seeded VLP-16 ray-cast sweeps, random planes+edges scenes; bags unavailable offline)",
        "config": {"workload": "config4: independent VLP-16 problems (SR prev+cur, odometry L-M, mapping L-M)",
                   "problems_per_gpu": B, "global_batch": world * B, "points_per_sweep": 28800,
                   "parallelism": f"shard{world}"},
        "roofline": roof,
        "roofline_kernels": roof_all,
        "cpu_baseline": cpu,
        "parity": parity,
        "kernel_ms_per_step": stage_ms,
        "single_stream": stream,
        "host_upload": {"ms": upload_s * 1e3, "pcie_inclusive_value": B / (upload_s + ms_per_step * 1e-3),
                        "note": "rank 0; pageable host sweeps packed and copied per sweep; not the metric"},
        "workload_stats": {"od_iters_mean": st["od_iters"] / B, "mp_iters_mean": st["mp_iters"] / B,
                           "mp_stack_mean": st["mp_stack"] / B, "mp_map_points_mean": st["mp_map_points"] / B,
                           "od_queries_mean": st["od_queries"] / B,
                           "mp_fit_fraction": st["mp_fits"] / max(st["mp_stack_iters"], 1)},
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
