"""Benchmark: scans/sec of the LOAM hot path (scan registration + odometry L-M + mapping L-M) on
MI355X, BASELINE.json config 4 shape: independent synthetic VLP-16 problems, sharded across ranks.

One step = one pass of the whole hot path over this rank's batch of problems, inputs resident in
HBM: scan registration of both sweeps of every problem, odometry seeded from prev and solved on
cur, mapping of prev into an empty map and solved for cur.  Sharding: contiguous
ranges of problems per rank (seeds 1000 + global index), no collective on the data path; one
all-gather of the poses after the timed steps.

  --split strong (default, the `value`): --global-batch problems in total (BASELINE config 4:
                 1024), global_batch / N per rank — a driver `--gpus N` run reports config 4 itself
  --split weak   (reported beside it in "weak", or as `value` when chosen): every rank owns
                 --batch problems (at N = 1 both splits are the same 1024 problems)

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--split weak|strong]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment the script launches the N ranks itself
(torch.distributed.run as a child process; the parent touches no GPU).  Ranks use RCCL ("nccl")
when a GPU is present, gloo otherwise (the CPU test harness).
"""
import argparse
import hashlib
import importlib
import json
import os
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# hardware queues per process (HIP's default is 4): the config-3 node pipeline runs three contexts
# with two streams each; with 4 queues streams of different nodes share a queue and serialise
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

METRIC = "scans/sec (odometry+mapping L-M solve) VLP-16 sweep, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# chip-wide rate of rows gathered from an XCD's L2 (MI355X_MICROARCH.md, "Indexed rows: gather into
# LDS": 16.8-18.8 TB/s): the ceiling of the search kernels, whose gathers hit L2, not HBM
L2_GATHER_PEAK_GBS = 16800.0
BASE_SEED = 1000


def shard(rank, world, batch, split, global_batch):
    """(first global problem index, problems) owned by `rank`: weak = `batch` per rank, strong =
    `global_batch` split into contiguous equal ranges"""
    if split == "weak":
        return rank * batch, batch
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} does not split over {world} ranks")
    per = global_batch // world
    return rank * per, per


def kernel_bytes(st):
    """Bytes each kernel moves over one step of the whole batch, split by the kernel that moves them
    (DESIGN.md §4).  Streaming kernels: the algorithmic bytes of SURVEY.md §8(d).  Search kernels
    (k_od_assoc, k_mp_nnfit): the bytes they actually gather, from the engine's work counters (cells,
    candidates, window points, chunk boxes), since their cost is the search, not the algorithmic
    16 B per query."""
    feats = 16 * (st["n_sharp"] + st["n_less_sharp"] + st["n_flat"] + st["n_less_flat"])
    return {
        "k_sr_ring_sort": 16 * st["n_raw"] + 16 * st["n_ring"],
        "k_sr_features": 16 * st["n_ring"],
        "k_sr_select": 16 * st["n_ring"] + feats,
        # per query and round: its point (16 B), 27 bucket bounds (8 B each), the three indices
        # written (12 B); plus every Last point (16 B) and chunk box (32 B) loaded
        "k_od_assoc": (16 + 27 * 8 + 12) * st["od_queries"] + 16 * st["od_assoc_gathered"]
                      + 32 * st["od_assoc_boxes"],
        # per iteration: every stored row's coefficient (16 B) + accept flag (1 B) read back (Q12:
        # all rows so far re-evaluated at the current transform), the query point read (16 B) and
        # its coefficient + flag written (17 B); with the per-query moments (tuning od_moments_min,
        # st["od_moments"]) the query point (16 B) and its ten fp64 moments read and written (160 B)
        "k_od_rows": (176 * st["od_query_iters"] if st.get("od_moments")
                      else 17 * st["od_row_evals"] + 33 * st["od_query_iters"]),
        # per query-iteration: accept flag, stack point and coefficient read back for JtJ
        "k_mp_iter": 33 * st["mp_stack_iters"],
        # the search and the fit in one launch, one 64-B record per query (last 5-NN + its fit): per
        # query-iteration the stack point (16 B), the record's 5-NN read (32 B) and its fit read (32 B,
        # an upper bound: only reused fits are read); per refit the 5 neighbours (80 B) and the record
        # written (64 B; a record is written only when its list changes, round 6); the rows stay in
        # the kernel (fused step); the search's 8 B per bucket range and 16 B per map point evaluated
        # (seeds included)
        "k_mp_nnfit": 80 * st["mp_stack_iters"] + 8 * st["mp_nn_cells"] + 16 * st["mp_nn_candidates"]
                      + 144 * st["mp_fits"],
    }


SEARCH_KERNELS = ("k_mp_nnfit", "k_od_assoc")


def algorithmic_bytes(st):
    """SURVEY.md §8(d)'s algorithmic bytes per kernel and step: what the kernel must read and write
    at minimum.  Equal to kernel_bytes for the streaming kernels.  The search and mapping L-M
    kernels are priced by B_MP's / B_OD's per-unit terms, not by the candidates the search visits or
    the engine's own caches (the MpFit record): k_mp_nnfit = per query-iteration the stack point and
    its 5 neighbours (16 + 80 B) and per accepted row 64 B (the row written and read back, B_MP's
    64 r_k; the mapping rows' counter mp_rows_sum); k_mp_iter's row reads are part of those 64 B, so it is not priced on its
    own; k_od_assoc = per association round every Last point once (16 B (C + S), B_OD)."""
    alg = dict(kernel_bytes(st))
    alg["k_mp_nnfit"] = 96 * st["mp_stack_iters"] + 64 * st["mp_rows_sum"]
    alg.pop("k_mp_iter")
    alg["k_od_assoc"] = 16 * st["od_assoc_points"]
    # the VoxelGrid jobs (B_MP's 32 s and 32 M_valid, MP-4 / MP-8): the stacks read every mapped
    # sweep's lessSharp + lessFlat point once (16 B) and write the downsampled stack (16 B per
    # point; the solved frame's stack, mp_stack: the first frame's output is not counted, a lower
    # bound); the cubes read and write the valid cubes' points (32 B per point of the solved
    # frame's valid cubes: the first frame's smaller map is not counted)
    alg["vg_stack"] = 16 * (st["n_less_sharp"] + st["n_less_flat"]) + 16 * st["mp_stack"]
    alg["vg_cubes"] = 32 * st["mp_map_valid_points"]
    return alg


def moved_od_bytes(st):
    """B_OD as the engine moves it: with the per-query moments (tuning od_moments_min) the stored
    rows are never re-read, so SURVEY.md §8(d)'s Σ 32 R_k term (Q12's row re-reads) is replaced
    by the moments' 176 B per query-iteration (query point 16 B + ten fp64 moments read and
    written, 160 B)"""
    if not st.get("od_moments"):
        return st["bytes_od"]
    return st["bytes_od"] - 32 * st["od_rows_sum"] + 176 * st["od_query_iters"]


# what bounds each kernel in practice: the roofline is priced against HBM, but the
# search kernels are limited by dependent gathers, not bandwidth
LIMITED_BY = {"k_od_assoc": "latency (dependent gathers)",
              "k_mp_nnfit": "latency (dependent gathers, then the fit's VALU)",
              "k_sr_select": "latency (serial greedy picks)"}


def load_traffic(traffic_file):
    """{kernel: PMC HBM bytes per launch} (profiles/traffic*.json, tools/pmc_traffic.py), or {}"""
    tpath = os.path.join(ROOT, "profiles", traffic_file)
    try:
        d = json.load(open(tpath))
    except Exception:
        return {}
    return {k: v for k, v in d.items() if isinstance(v, (int, float))}


def rooflines(st, st_prof, ktimes, psteps, ms_per_step, traffic_file="traffic.json"):
    """(roofline of the dominant kernel, every kernel's, the whole step's, ms per step per kernel)
    from one workload's work counters (st: the timed steps; st_prof: the profiling pass, whose
    search-kernel counters kernel_bytes needs) and its per-kernel HIP-event times (ktimes: name ->
    (total ms, launches) over psteps steps)"""
    # roofline of the dominant kernel: bytes per launch / average launch duration
    kb = kernel_bytes(st_prof)
    alg_kb = algorithmic_bytes(st_prof)
    priced = {k: v for k, v in ktimes.items() if k in alg_kb}
    dom = max(priced.items(), key=lambda kv: kv[1][0])[0] if priced else None
    roof = None
    tmap = load_traffic(traffic_file)
    if dom:
        tot_ms, launches = ktimes[dom]
        avg_ms = tot_ms / max(launches, 1)
        launches_per_step = launches / psteps
        traffic = tmap.get(dom)
        alg_launch = alg_kb[dom] / launches_per_step
        achieved = alg_launch / (avg_ms * 1e-3) / 1e9
        roof = {"kernel": dom, "bound": "hbm", "limited_by": LIMITED_BY.get(dom, "hbm"),
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic, "avg_launch_ms": avg_ms, "bytes_per_launch": alg_launch,
                "bytes_model": "algorithmic bytes, SURVEY.md §8(d) per-unit figure x units (bench.algorithmic_bytes)"}
        if traffic:
            roof["traffic_gbs"] = traffic / (avg_ms * 1e-3) / 1e9
            roof["traffic_frac"] = roof["traffic_gbs"] / HBM_PEAK_GBS
            # HBM bytes (PMC, profiles/traffic*.json) per algorithmic byte: > 1 = re-reads / engine caches
            roof["traffic_over_algorithmic"] = traffic / alg_launch
        if dom in SEARCH_KERNELS:
            # what the search actually reads (candidate cells, window points, chunk boxes), from the
            # work counters: L2-resident gathers, priced against the chip's L2 gather rate
            g_launch = kb[dom] / launches_per_step
            g = g_launch / (avg_ms * 1e-3) / 1e9
            roof["gathered"] = {"bytes_per_launch": g_launch, "achieved_gbs": g,
                                "l2_gather_peak": L2_GATHER_PEAK_GBS, "l2_frac": g / L2_GATHER_PEAK_GBS}
    stage_ms = {k: round(v[0] / psteps, 4) for k, v in sorted(ktimes.items())}
    roof_all = {}
    for k, nbytes in alg_kb.items():
        if k in ktimes and ktimes[k][0] > 0:
            sec = ktimes[k][0] / psteps * 1e-3
            gbs = nbytes / sec / 1e9  # algorithmic bytes per step / s per step
            roof_all[k] = {"achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                           "ms_per_step": round(ktimes[k][0] / psteps, 4),
                           "bytes_per_step": int(nbytes), "limited_by": LIMITED_BY.get(k, "hbm")}
            if k in tmap and nbytes > 0:  # PMC HBM bytes (per launch x launches per step) / algorithmic
                t_step = tmap[k] * ktimes[k][1] / psteps
                roof_all[k]["traffic_per_step"] = int(t_step)
                roof_all[k]["traffic_over_algorithmic"] = round(t_step / nbytes, 3)
            if k in SEARCH_KERNELS:
                ggbs = kb[k] / sec / 1e9
                roof_all[k]["gathered"] = {"bytes_per_step": int(kb[k]), "achieved_gbs": round(ggbs, 1),
                                           "l2_frac": round(ggbs / L2_GATHER_PEAK_GBS, 4)}
    # the whole pipeline against HBM: the algorithmic bytes the engine's path moves per step / step
    # time (B_SR + B_OD + B_MP; B_OD in its moments form when the odometry keeps them, which moves no
    # stored rows), with SURVEY.md §8(d)'s literal figure (the Q12 row re-reads) beside it
    alg = int(st["bytes_sr"] + moved_od_bytes(st) + st["bytes_mp"])
    survey = int(st["bytes_sr"] + st["bytes_od"] + st["bytes_mp"])
    sec = ms_per_step * 1e-3
    pipeline = {"algorithmic_bytes_per_step": alg, "achieved_gbs": alg / sec / 1e9,
                "frac": alg / sec / 1e9 / HBM_PEAK_GBS,
                "bytes_model": ("B_SR + B_OD + B_MP per step (SURVEY.md §8(d)); B_OD's stored-row term "
                                "as moved: " + ("176 B per query-iteration (per-query moments)"
                                                if st.get("od_moments") else "32 R_k (rows re-read)")),
                "survey_literal": {"bytes_per_step": survey, "frac": survey / sec / 1e9 / HBM_PEAK_GBS,
                                   "note": "B_OD with Sigma 32 R_k, the row re-reads the reference's Q12 implies"},
                "kernel_busy_ms_per_step": round(sum(v[0] for v in ktimes.values()) / psteps, 4) if ktimes else None}
    return roof, roof_all, pipeline, stage_ms


def uses_moments(eng, P):
    """whether the engine's odometry keeps the stored rows as per-query moments at batch size P
    (tuning od_moments_min; the rows kernel's byte model depends on it)"""
    get = getattr(eng, "get_tuning", None)
    if get is None:
        return False
    return P > get("od_small_max") and P >= get("od_moments_min")


def stream_leg(loam, sg, n_sweeps, n_cpu, stages=3, priority="default", tune=None, reps=3):
    """Config 3 (streaming, seed 1): scan registration -> odometry -> mapping on every published
    frame, one sweep at a time on one GPU context, next to the CPU oracle on the first sweeps.
    Each mode runs `reps` times on fresh contexts (the same 220 sweeps from the start); the median
    time is reported with every run's (these latency-bound legs vary by +-5-10 % from run to run)."""
    sweeps = sg.stream_sweeps(n_sweeps, 1)

    def Eng(cfg=None):  # (tune: launch choices of the A/B runs)
        e = loam.Engine(cfg)
        if tune:
            e.set_tuning(**tune)
        return e

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

    def median_runs(once):
        """(poses of the first run, sweeps, median seconds, every run's ms per sweep)"""
        res = [once() for _ in range(max(1, reps))]
        ts = sorted(r[2] for r in res)
        n = res[0][1]
        return res[0][0], n, ts[len(ts) // 2], [round(1e3 * r[2] / max(n, 1), 4) for r in res]

    def fresh_seq():
        e = Eng(loam.default_config())
        r = run(e, sweeps)
        e.close()
        return r

    warm = Eng(loam.default_config(system_delay=1))
    run(warm, sweeps[:6])
    warm.close()
    pg, ng, tg, runs_seq = median_runs(fresh_seq)
    out = {"config": f"config3: VLP-16 stream (seed 1), {n_sweeps} sweeps, systemDelay 20, mapping every 2nd frame",
           "sweeps_processed": ng, "scans_per_s": ng / tg, "ms_per_sweep": 1e3 * tg / max(ng, 1),
           "runs_ms_per_sweep": runs_seq,
           "mode": "sequential: one thread calls the three node bodies in turn on one context (per-sweep latency)"}

    # the same sweeps through loam_chain_sweep: the three bodies on one context with the
    # intermediate topics left in device memory (intra-process / nodelet deployment)
    def run_chain(eng, sw):
        poses, n, t = [], 0, 0.0
        for k, s in enumerate(sw):
            a = time.perf_counter()
            rc, pub, od, aft, bef, _ = eng.chain_sweep(s, stamp=0.1 * k)
            if rc == 0:
                n += 1
                if aft is not None:
                    poses.append(aft)
            t += time.perf_counter() - a
        return np.array(poses), n, t

    def fresh_chain():
        e = Eng(loam.default_config())
        r = run_chain(e, sweeps)
        e.close()
        return r

    warm_c = Eng(loam.default_config(system_delay=1))
    run_chain(warm_c, sweeps[:6])
    warm_c.close()
    pc, nc, tc_, runs_chain = median_runs(fresh_chain)
    out["device_chain"] = {"mode": "sequential, intermediate topics left on the device (loam_chain_sweep)",
                           "sweeps_processed": nc, "scans_per_s": nc / tc_, "ms_per_sweep": 1e3 * tc_ / max(nc, 1),
                           "runs_ms_per_sweep": runs_chain,
                           "max_abs_err_vs_sequential": float(np.abs(pc - pg).max()) if pc.shape == pg.shape else None}

    # the same sweeps through the node pipeline (loam_velodyne-1_amd/pipeline.py): one context and
    # one thread per node, as the reference's node processes run; outputs must equal the sequential run
    pl_mod = importlib.import_module("loam_velodyne-1_amd.pipeline")
    warm_pl = pl_mod.NodePipeline(Eng, loam.default_config(system_delay=1), stages=stages)
    warm_pl.run(sweeps[:6])
    warm_pl.close()
    if priority == "default":
        priority = pl_mod.NodePipeline.DEFAULT_PRIORITY
    busy = []

    def fresh_pipe():
        pl = pl_mod.NodePipeline(Eng, loam.default_config(), stages=stages, priority=priority)
        a = time.perf_counter()
        res, n_pl = pl.run(sweeps)
        t_pl = time.perf_counter() - a
        busy.append(dict(pl.busy_s))
        pl.close()
        return np.array([r[0] for r in res]), n_pl, t_pl

    pp, n_pl, t_pl, runs_pipe = median_runs(fresh_pipe)
    out["pipelined"] = {"mode": "node pipeline: scanRegistration / laserOdometry / laserMapping on three "
                                "contexts and three threads (reference: separate node processes)",
                        "sweeps_processed": n_pl, "scans_per_s": n_pl / t_pl, "ms_per_sweep": 1e3 * t_pl / max(n_pl, 1),
                        "runs_ms_per_sweep": runs_pipe,
                        "node_busy_ms_per_sweep": {k: round(1e3 * v / max(n_pl, 1), 4) for k, v in busy[0].items()},
                        "max_abs_err_vs_sequential": float(np.abs(pp - pg).max()) if pp.shape == pg.shape else None}
    if n_cpu > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as oc
        with pinned_core() as core:
            po, no, tc = run(oc.Oracle(oc.default_config()), sweeps[:n_cpu])
        k = min(len(po), len(pg))
        out["cpu_oracle"] = {"sweeps_processed": no, "scans_per_s": no / tc, "cores": 1, "kind": "port",
                             "pinned_cpu": core}
        out["speedup_vs_cpu"] = out["scans_per_s"] / out["cpu_oracle"]["scans_per_s"]
        out["device_chain"]["speedup_vs_cpu"] = out["device_chain"]["scans_per_s"] / out["cpu_oracle"]["scans_per_s"]
        out["pipelined"]["speedup_vs_cpu"] = out["pipelined"]["scans_per_s"] / out["cpu_oracle"]["scans_per_s"]
        out["max_abs_err_mapping"] = float(np.abs(pg[:k] - po[:k]).max()) if k else None
    return out


def latency_leg(loam, sg, runs, warmup, seed=0, lidar=None, cfg=None,
                config="config2: one VLP-16 problem (seed 0), warm context, inputs resident"):
    """Config 2 (and config 5 with lidar=HDL64): one problem (prev, cur) at a time, warm (context and
    buffers reused), the whole problem on the device per call; ms per problem (median of `runs`)"""
    prev, cur = sg.single_problem(seed) if lidar is None else sg.single_problem(seed, lidar=lidar)
    eng = loam.Engine(cfg) if cfg is not None else loam.Engine()
    eng.batch_upload([prev], [cur])
    for _ in range(warmup):
        eng.batch_run()
        eng.sync()
    ts = []
    for _ in range(runs):
        a = time.perf_counter()
        eng.batch_run()
        eng.sync()
        ts.append(time.perf_counter() - a)
    od, aft, _ = eng.batch_download()
    eng.close()
    return {"config": config,
            "ms_median": 1e3 * statistics.median(ts), "ms_min": 1e3 * min(ts), "runs": runs}, (prev, cur, od, aft)


class pinned_core:
    """pin the calling thread to one core for the CPU baseline (taskset -c 0)"""

    def __enter__(self):
        self.old = os.sched_getaffinity(0)
        self.core = min(self.old)
        os.sched_setaffinity(0, {self.core})
        return self.core

    def __exit__(self, *a):
        os.sched_setaffinity(0, self.old)


def cpu_leg(oc, prevs, curs, od, aft, n_sample, reps, ocfg=None):
    """The oracle (single-thread C++ restatement), pinned to one core, over a bounded sample of the
    batch's problems spread across it: 1 warm-up run, then the median of `reps` runs (BASELINE.md
    §2).  Also checks the engine's poses of the sampled problems against the oracle.  ocfg: the
    oracle's configuration (default: the VLP-16 one)"""
    B = len(prevs)
    idx = sorted(set(int(round(v)) for v in np.linspace(0, B - 1, min(n_sample, B))))
    times = []
    err_od = err_mp = 0.0
    with pinned_core() as core:
        for r in range(reps + 1):
            a = time.perf_counter()
            outs = [oc.problem(prevs[i], curs[i]) if ocfg is None else oc.problem(prevs[i], curs[i], ocfg)
                    for i in idx]
            t = time.perf_counter() - a
            if r == 0:
                for i, (od_o, aft_o, _) in zip(idx, outs):
                    err_od = max(err_od, float(np.abs(od[i] - od_o).max()))
                    err_mp = max(err_mp, float(np.abs(aft[i] - aft_o).max()))
            else:
                times.append(t)
    med = statistics.median(times)
    model = "unknown CPU"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cpu = {"value": len(idx) / med, "unit": "scans/s", "cores": 1, "kind": "port",
           "sample": f"{len(idx)} problems spread over the batch (global indices {idx[0]}..{idx[-1]}), "
                     f"oracle/liboracle.so -O3, one thread pinned to CPU {core} of {model} "
                     f"({os.cpu_count()} logical CPUs visible); median of {reps} runs after 1 warm-up, "
                     f"{med:.2f} s per run (runs: {', '.join(f'{t:.2f}' for t in times)})"}
    parity = {"problems_checked": len(idx), "max_abs_err_odometry": err_od, "max_abs_err_mapping": err_mp}
    return cpu, parity


# config 5 (BASELINE.json: dense HDL-64E sweeps, the HBM roofline stress) with the reference's
# 64-ring settings: linear ring model, 100 odometry / 20 mapping iterations
# (bk include/loam_velodyne/common.h:26-32, src/scanRegistration.cpp:268-275)
DENSE_CFG = dict(n_rings=64, max_points=160000, od_max_iter=100, mp_max_iter=20)
DENSE_SEED = 5000


def dense_batch_leg(loam, sg, B, steps, warmup, profile_steps, cpu_sample, cpu_reps, device=0, tune=None):
    """Config 5 as a batch: B independent HDL-64E problems (seeds DENSE_SEED + i, ~131k points per
    sweep, 64 rings) through the same step as config 4 — enough sweeps in flight to load the chip,
    which one 131k-point problem does not.  Inputs resident in HBM; its own roofline (dominant kernel
    and whole step), CPU oracle sample and parity."""
    prevs, curs = sg.batch_problems(B, base_seed=DENSE_SEED, lidar=sg.HDL64)
    eng = loam.Engine(loam.default_config(ring_model=loam.RING_LINEAR, **DENSE_CFG), device=device)
    if tune:
        eng.set_tuning(**tune)
    eng.batch_upload(prevs, curs)
    elapsed = timed(eng, steps, warmup, None, "cpu")
    od, aft, st = eng.batch_download()
    ms = elapsed / steps * 1e3
    ktimes, st_prof = {}, st
    if profile_steps > 0:
        eng.set_profiling(True)
        for _ in range(profile_steps):
            eng.batch_run()
        _, _, st_prof = eng.batch_download()
        ktimes = eng.kernel_times()
        eng.set_profiling(False)
    st["od_moments"] = st_prof["od_moments"] = uses_moments(eng, B)
    eng.close()
    roof, roof_all, pipeline, stage_ms = rooflines(st, st_prof, ktimes, max(profile_steps, 1), ms,
                                                   traffic_file="traffic_config5.json")
    out = {"config": f"config5 batch: {B} HDL-64E problems (seeds {DENSE_SEED}..{DENSE_SEED + B - 1}, 64 rings, "
                     "linear ring model, 100 / 20 iterations), inputs resident",
           "problems": B, "points_per_sweep_mean": float(np.mean([len(c) for c in curs])),
           "value": B * steps / elapsed, "unit": "scans/s", "ms_per_step": ms, "steps": steps, "warmup": warmup,
           "roofline": roof, "roofline_kernels": roof_all, "pipeline": pipeline, "kernel_ms_per_step": stage_ms,
           "workload_stats": {"od_iters_mean": st["od_iters"] / B, "mp_iters_mean": st["mp_iters"] / B,
                              "mp_stack_mean": st["mp_stack"] / B, "od_queries_mean": st["od_queries"] / B}}
    if cpu_sample > 0 and not os.environ.get("LOAM_BENCH_ENGINE"):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as oc
        cpu, parity = cpu_leg(oc, prevs, curs, od, aft, cpu_sample, cpu_reps,
                              ocfg=oc.default_config(ring_model=1, **DENSE_CFG))
        out["cpu_baseline"] = cpu
        out["parity"] = parity
        out["speedup_vs_cpu"] = out["value"] / cpu["value"]
    return out


def engine_factory(tune=None):
    """the engine under measurement: libloam_hip.so through its ctypes binding.  LOAM_BENCH_ENGINE
    ("module:attr") substitutes a stand-in for the harness tests on CPU-only machines (gloo);
    it is never set for a measurement.  tune: {key: value} launch choices (loam_set_tuning), for A/B
    runs of the same library."""
    spec = os.environ.get("LOAM_BENCH_ENGINE")
    if spec:
        mod, attr = spec.split(":")
        return getattr(importlib.import_module(mod), attr)
    E = importlib.import_module("loam_velodyne-1_amd").Engine
    if not tune:
        return E

    def make(*a, **k):
        e = E(*a, **k)
        e.set_tuning(**tune)
        return e
    return make


def parse_tune(items):
    out = {}
    for it in items or []:
        k, v = it.split("=")
        out[k.strip()] = int(v)
    return out


def timed(eng, steps, warmup, dist, sync_dev):
    """W untimed steps, then exactly K steps between barrier + sync; the max over ranks (s)"""
    for _ in range(warmup):
        eng.batch_run()
    eng.sync()
    if dist:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.batch_run()
    eng.sync()
    elapsed = time.perf_counter() - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=sync_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    return elapsed


def fed_leg(Engine, sg, prevs, curs, steps, warmup, device):
    """Batches arriving over time: each step's sweeps handed over from host memory with
    loam_batch_feed (pack into pinned staging + PCIe copy on the pipeline's stream, inside the timed
    region), alternating two distinct batches of the same size, so no step re-runs the previous
    step's inputs; and the resident batch with the step pipeline off (step_pipe = sr_ahead = 0:
    each step's stages in sequence, no work enqueued ahead).  Reported beside the metric, which
    times the resident batch through the pipeline."""
    B = len(prevs)
    prevs2, curs2 = sg.batch_problems(B, base_seed=BASE_SEED + 100000)
    out = {}
    loam = importlib.import_module("loam_velodyne-1_amd")
    # (measured: the same sweeps from caller memory registered with hipHostRegister and copied per
    # sweep without the staging pack ran at 89 ms/step against 43: the pack into hipHostMalloc'd
    # staging stays)

    def run_fed(fb):
        eng = Engine(device=device)
        eng.batch_upload(prevs, curs)
        for k in range(warmup):
            eng.batch_feed(fb[k % 2])
            eng.batch_run()
        eng.sync()
        t0 = time.perf_counter()
        for k in range(steps):
            eng.batch_feed(fb[k % 2])
            eng.batch_run()
        eng.sync()
        el = time.perf_counter() - t0
        eng.close()
        return el

    E = loam.Engine  # (prepare_batch: a static helper of the binding)
    el = run_fed([E.prepare_batch(prevs, curs), E.prepare_batch(prevs2, curs2)])
    out["fed_from_host"] = {"value": B * steps / el, "ms_per_step": el / steps * 1e3, "problems": B,
                            "note": "every step's sweeps fed from pageable host memory (loam_batch_feed: "
                                    "pack into pinned staging + PCIe copy inside the timed region), two "
                                    "distinct batches alternating"}
    e2 = Engine(device=device)
    e2.set_tuning(step_pipe=0, sr_ahead=0)
    e2.batch_upload(prevs, curs)
    el2 = timed(e2, steps, warmup, None, "cpu")
    e2.close()
    out["unpipelined"] = {"value": B * steps / el2, "ms_per_step": el2 / steps * 1e3, "problems": B,
                          "note": "inputs resident, step_pipe = sr_ahead = 0: no stage of a step "
                                  "overlaps another step's"}
    return out


def gather_poses(dist, od, aft, world, dev):
    """the one collective of the sharded path: every rank's (odometry, mapping) poses, in global
    problem order (RCCL all-gather on GPUs)"""
    import torch
    mine = torch.from_numpy(np.concatenate([od, aft], axis=1).astype(np.float32)).to(dev)
    if dev == "cpu":  # gloo
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        return torch.cat(parts).numpy()
    allp = torch.empty((world * mine.shape[0], 12), dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(allp, mine)
    return allp.cpu().numpy()


def spawn(args_list, n):
    """launch n ranks of this script (torch.distributed.run) as a child; returns its exit code"""
    port = os.environ.get("MASTER_PORT", "29511")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__)] + args_list
    return subprocess.call(cmd)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU (weak split)")
    ap.add_argument("--global-batch", type=int, default=1024, help="problems in total (strong split)")
    ap.add_argument("--split", choices=("weak", "strong"), default="strong", help="which split is `value`")
    ap.add_argument("--strong-leg", type=int, default=1, help="also measure the other split (0: skip)")
    ap.add_argument("--cpu-sample", type=int, default=32, help="problems in the CPU baseline sample (0: skip)")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--stream-sweeps", type=int, default=220, help="config-3 streaming leg (0: skip)")
    ap.add_argument("--stream-cpu-sweeps", type=int, default=220, help="CPU oracle over the same sweeps as the GPU legs")
    ap.add_argument("--latency-runs", type=int, default=50, help="config-2 warm latency leg (0: skip)")
    ap.add_argument("--dense-batch", type=int, default=64, help="config-5 batched HDL-64E leg: problems (0: skip)")
    ap.add_argument("--dense-steps", type=int, default=5)
    ap.add_argument("--dense-cpu-sample", type=int, default=2)
    ap.add_argument("--tune", action="append", default=[], help="key=value launch choice (loam_set_tuning), repeatable")
    ap.add_argument("--fed-leg", type=int, default=1, help="fed-from-host and unpipelined legs at N = 1 (0: skip)")
    ap.add_argument("--share-only", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--dense-only", type=int, default=0, help="run only the config-5 batched leg (profiling)")
    argv = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(argv)
    tune = parse_tune(args.tune)

    if args.share_only:  # child: the 8-GPU share timed alone in a fresh process, as one rank runs it
        first, B8 = shard(0, 8, args.batch, "strong", args.global_batch)
        prevs, curs = importlib.import_module("loam_velodyne-1_amd.synthgen").batch_problems(B8, base_seed=BASE_SEED + first)
        e8 = engine_factory(tune)(device=0)
        e8.batch_upload(prevs, curs)
        el = timed(e8, args.steps, args.warmup, None, "cpu")
        e8.close()
        print(json.dumps({"problems": B8, "value": B8 * args.steps / el, "ms_per_step": el / args.steps * 1e3}))
        return

    if args.dense_only:  # the config-5 batched leg alone (rocprof passes of tools/profile.sh)
        loam = importlib.import_module("loam_velodyne-1_amd")
        sg = importlib.import_module("loam_velodyne-1_amd.synthgen")
        print(json.dumps(dense_batch_leg(loam, sg, args.dense_batch, args.dense_steps, 2, args.profile_steps,
                                         args.dense_cpu_sample if args.cpu_sample > 0 else 0, 3, tune=tune)))
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(argv, args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist, dev = None, "cpu"
    if world > 1:
        import torch
        import torch.distributed as tdist
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            dev = f"cuda:{local}"
            tdist.init_process_group("nccl")
        else:  # CPU-only harness test
            tdist.init_process_group("gloo")
        dist = tdist

    share8 = None
    if args.strong_leg and world == 1 and args.global_batch % 8 == 0:
        # the per-GPU share of config 4 on 8 GPUs (1024 / 8), measured on one GPU in a child process
        # started before this one touches the GPU: a fresh process, as each of the 8 ranks is (timed
        # in this process after the batch-1024 leg it measured ~10 % slower)
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--share-only", "1", "--steps", str(args.steps),
                              "--warmup", str(args.warmup), "--batch", str(args.batch),
                              "--global-batch", str(args.global_batch)] + [f"--tune={t}" for t in args.tune],
                             capture_output=True, text=True)
        if out.returncode != 0:
            raise SystemExit(f"8-GPU share child failed ({out.returncode}): {out.stderr[-2000:]}")
        share8 = json.loads(out.stdout.strip().splitlines()[-1])

    Engine = engine_factory(tune)
    sg = importlib.import_module("loam_velodyne-1_amd.synthgen")

    def leg(split):
        first, B = shard(rank, world, args.batch, split, args.global_batch)
        prevs, curs = sg.batch_problems(B, base_seed=BASE_SEED + first)
        eng = Engine(device=local)
        eng.batch_upload(prevs, curs)
        elapsed = timed(eng, args.steps, args.warmup, dist, dev)
        od, aft, st = eng.batch_download()
        return {"first": first, "B": B, "prevs": prevs, "curs": curs, "eng": eng, "elapsed": elapsed,
                "od": od, "aft": aft, "st": st}

    main_leg = leg(args.split)
    other = None
    same = shard(rank, world, args.batch, "weak", args.global_batch) == \
        shard(rank, world, args.batch, "strong", args.global_batch)
    if args.strong_leg and same:  # the other split is this very workload (N = 1, batch = global batch)
        other = {"split": "strong" if args.split == "weak" else "weak", "global_batch": world * main_leg["B"],
                 "problems_per_gpu": main_leg["B"], "value": world * main_leg["B"] * args.steps / main_leg["elapsed"],
                 "ms_per_step": main_leg["elapsed"] / args.steps * 1e3, "note": "same workload as value"}
    elif args.strong_leg:
        other_split = "strong" if args.split == "weak" else "weak"
        o = leg(other_split)
        o["eng"].close()
        other = {"split": other_split, "global_batch": world * o["B"], "problems_per_gpu": o["B"],
                 "value": world * o["B"] * args.steps / o["elapsed"], "ms_per_step": o["elapsed"] / args.steps * 1e3}
    if share8 is not None:
        other["one_gpu_at_8gpu_share"] = share8

    eng, B, elapsed, st = main_leg["eng"], main_leg["B"], main_leg["elapsed"], main_leg["st"]
    od, aft = main_leg["od"], main_leg["aft"]

    fed = None
    if args.fed_leg and world == 1 and not os.environ.get("LOAM_BENCH_ENGINE"):
        fed = fed_leg(Engine, sg, main_leg["prevs"], main_leg["curs"], args.steps, args.warmup, local)

    # host-buffer rate: the same batch handed over from host memory, upload + one step
    a = time.perf_counter()
    eng.batch_upload(main_leg["prevs"], main_leg["curs"])
    eng.sync()
    upload_s = time.perf_counter() - a

    # per-kernel device times of the same workload (HIP events on the engine stream), untimed
    # (the profiling pass also runs the search kernels' counting variants: their work counters, which
    # kernel_bytes needs, come from this pass, st_prof)
    ktimes, st_prof = {}, st
    if args.profile_steps > 0:
        eng.set_profiling(True)
        for _ in range(args.profile_steps):
            eng.batch_run()
        _, _, st_prof = eng.batch_download()
        ktimes = eng.kernel_times()
        eng.set_profiling(False)

    gathered = None
    if dist:
        gathered = gather_poses(dist, od, aft, world, dev)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed
    psteps = max(args.profile_steps, 1)

    st["od_moments"] = st_prof["od_moments"] = uses_moments(eng, B)
    roof, roof_all, pipeline, stage_ms = rooflines(st, st_prof, ktimes, psteps, ms_per_step)

    # CPU baseline: the oracle on a bounded sample, N=1 only
    cpu = parity = None
    if world == 1 and args.cpu_sample > 0 and not os.environ.get("LOAM_BENCH_ENGINE"):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as oc
        cpu, parity = cpu_leg(oc, main_leg["prevs"], main_leg["curs"], od, aft, args.cpu_sample, args.cpu_reps)

    stream = latency = None
    if world == 1 and not os.environ.get("LOAM_BENCH_ENGINE"):
        loam = importlib.import_module("loam_velodyne-1_amd")
        if args.stream_sweeps > 0:
            stream = stream_leg(loam, sg, args.stream_sweeps, args.stream_cpu_sweeps, tune=tune)
        if args.latency_runs > 0:
            def with_cpu(lat, p0, c0, od0, aft0, ocfg=None):
                """the pinned oracle on the same problem: median of 3 after a warm-up, and the parity"""
                if args.cpu_sample > 0:
                    sys.path.insert(0, os.path.join(ROOT, "oracle"))
                    import oracle_ctypes as oc
                    with pinned_core():
                        ts = []
                        for _ in range(4):
                            a = time.perf_counter()
                            od_o, aft_o, _ = oc.problem(p0, c0) if ocfg is None else oc.problem(p0, c0, ocfg(oc))
                            ts.append(time.perf_counter() - a)
                    cpu_ms = 1e3 * statistics.median(ts[1:])
                    lat["cpu_oracle_ms"] = cpu_ms
                    lat["speedup_vs_cpu"] = cpu_ms / lat["ms_median"]
                    lat["max_abs_err"] = float(max(np.abs(od0[0] - od_o).max(), np.abs(aft0[0] - aft_o).max()))
                return lat

            latency, prob = latency_leg(loam, sg, args.latency_runs, 5)
            latency = with_cpu(latency, *prob)
            # config 5: one dense HDL-64E problem (64 rings, ~131k points per sweep)
            # (the reference's 64-ring settings: linear ring model, 100 odometry / 20 mapping iterations)
            dense_cfg = dict(n_rings=64, max_points=160000, od_max_iter=100, mp_max_iter=20)
            dense, prob = latency_leg(loam, sg, max(args.latency_runs // 5, 3), 2, seed=2, lidar=sg.HDL64,
                                      cfg=loam.default_config(ring_model=loam.RING_LINEAR, **dense_cfg),
                                      config="config5: one HDL-64E problem (seed 2, 64 rings), warm context, "
                                             "inputs resident")
            dense["points_per_sweep"] = int(len(prob[1]))
            latency["config5"] = with_cpu(dense, *prob, ocfg=lambda oc: oc.default_config(ring_model=1, **dense_cfg))
    dense = None
    if world == 1 and args.dense_batch > 0 and not os.environ.get("LOAM_BENCH_ENGINE"):
        loam = importlib.import_module("loam_velodyne-1_amd")
        dense = dense_batch_leg(loam, sg, args.dense_batch, args.dense_steps, 2, min(args.profile_steps, 2),
                                args.dense_cpu_sample if args.cpu_sample > 0 else 0, 3, device=local, tune=tune)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak" if args.split == "weak" else "strong",
        "vs_baseline": None,
        "dtype": "fp32 (fp64 JtJ accumulation)",
        "data": "synthetic (seeded VLP-16 ray-cast sweeps, random planes+edges scenes; bags unavailable offline)",
        "config": {"workload": "config4: independent VLP-16 problems (SR prev+cur, odometry L-M, mapping L-M)",
                   "problems_per_gpu": B, "global_batch": world * B, "points_per_sweep": 28800,
                   "split": args.split, "parallelism": f"shard{world}",
                   "step_overlap": ("consecutive steps run as a software pipeline (tuning step_pipe, P >= 64): "
                                    "step k's odometry beside step k-1's mapping, step k+1's scan "
                                    "registration + odometry seed enqueued ahead; the K timed steps "
                                    "contain exactly K of each stage (loam_batch_sync waits for all "
                                    "streams, including the stage enqueued ahead); the timed steps re-run "
                                    "the resident batch — arriving_batches gives fresh batches fed from "
                                    "the host each step and the pipeline-off rate"),
                   **({"tuning": tune} if tune else {})},
        "roofline": roof,
        "roofline_kernels": roof_all,
        "pipeline": pipeline,
        "cpu_baseline": cpu,
        "parity": parity,
        "strong" if args.split == "weak" else "weak": other,
        "kernel_ms_per_step": stage_ms,
        "arriving_batches": fed,
        "single_stream": stream,
        "latency": latency,
        "dense_batch": dense,
        "gathered": {"problems": int(gathered.shape[0]),
                     "sha1": hashlib.sha1(np.ascontiguousarray(gathered, np.float32).tobytes()).hexdigest()}
        if gathered is not None else None,
        "host_upload": {"ms": upload_s * 1e3, "pcie_inclusive_value": B / (upload_s + ms_per_step * 1e-3),
                        "note": "rank 0; pageable host sweeps packed and copied per sweep; not the metric"},
        "workload_stats": {"od_iters_mean": st["od_iters"] / B, "mp_iters_mean": st["mp_iters"] / B,
                           "mp_stack_mean": st["mp_stack"] / B, "mp_map_points_mean": st["mp_map_points"] / B,
                           "od_queries_mean": st["od_queries"] / B,
                           "mp_fit_fraction": st["mp_fits"] / max(st["mp_stack_iters"], 1),
                           "mp_nn_candidates_per_query": st_prof["mp_nn_candidates"] / max(st["mp_stack_iters"], 1),
                           "mp_nn_cells_per_query": st_prof["mp_nn_cells"] / max(st["mp_stack_iters"], 1),
                           "od_assoc_points_per_query": st_prof["od_assoc_gathered"] / max(st["od_queries"], 1),
                           "od_assoc_boxes_per_query": st_prof["od_assoc_boxes"] / max(st["od_queries"], 1)},
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
