"""Synthetic input determinism and the multi-rank sharding of bench.py (gloo, world size 2): the
tests call bench.py's own shard function and run bench.py itself with two ranks."""
import os
import socket

import numpy as np
import pytest


def test_generator_deterministic(sg):
    a = sg.single_problem(0)
    b = sg.single_problem(0)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    p1, c1 = sg.batch_problems(3, base_seed=1000)
    p2, c2 = sg.batch_problems(3, base_seed=1000)
    for x, y in zip(p1 + c1, p2 + c2):
        np.testing.assert_array_equal(x, y)


def test_vlp16_geometry(sg):
    prev, cur = sg.single_problem(0)
    assert cur.shape == (28800, 4)                 # 1800 azimuth steps x 16 lasers, every ray hits
    assert np.all(np.bincount(cur[:, 3].astype(int)) == 1800)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_ranges():
    import bench
    # weak: B per rank, contiguous, seeds 1000 + global index
    assert [bench.shard(r, 4, 1024, "weak", 1024) for r in range(4)] == [(0, 1024), (1024, 1024), (2048, 1024),
                                                                        (3072, 1024)]
    # strong: config 4's 1024 problems split 1024 / N: 128 per GPU on 8 GPUs
    s8 = [bench.shard(r, 8, 1024, "strong", 1024) for r in range(8)]
    assert s8 == [(128 * r, 128) for r in range(8)]
    assert sum(n for _, n in s8) == 1024
    with pytest.raises(ValueError):
        bench.shard(0, 3, 1024, "strong", 1024)


def _run_bench(args, env_extra):
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    env.update(env_extra)
    env["PYTHONPATH"] = os.path.join(ROOT, "tests") + os.pathsep + env.get("PYTHONPATH", "")
    env["LOAM_BENCH_ENGINE"] = "bench_stub:Engine"
    env["MASTER_PORT"] = str(_free_port())
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    return json.loads(lines[0])


def _expected_sha(sg, first, n):
    import hashlib
    import bench_stub
    prevs, curs = sg.batch_problems(n, base_seed=1000 + first)
    rows = [np.concatenate(bench_stub.poses_of(p, c)) for p, c in zip(prevs, curs)]
    return hashlib.sha1(np.ascontiguousarray(np.stack(rows), np.float32).tobytes()).hexdigest()


@pytest.mark.parametrize("split", ["weak", "strong"])
def test_bench_spawns_two_ranks_gloo(sg, split):
    """`python bench.py --gpus 2` (no torchrun in front) launches two ranks itself; on a CPU-only
    machine they use gloo.  One JSON line from rank 0 with n_gpus 2; the gathered poses are the
    global problems in order (checked against a single-process run of the same stand-in engine)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    out = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "3", "--global-batch", "4",
                      "--split", split, "--profile-steps", "1"], {})
    assert out["n_gpus"] == 2
    assert out["scaling"] == split
    per, other_per = (3, 2) if split == "weak" else (2, 3)
    assert out["config"]["problems_per_gpu"] == per and out["config"]["global_batch"] == 2 * per
    assert out["gathered"]["problems"] == 2 * per
    assert out["gathered"]["sha1"] == _expected_sha(sg, 0, 2 * per)
    other = out["strong" if split == "weak" else "weak"]
    assert other["global_batch"] == 2 * other_per and other["problems_per_gpu"] == other_per
    assert out["value"] > 0 and out["roofline"]["kernel"] == "k_mp_nnfit"


def test_bench_single_gpu_share_child(sg):
    """At N = 1 the per-GPU share of 8 GPUs (global batch / 8) is timed in a child process started
    before the parent touches the device, as one of the 8 ranks would run it; its line lands in the
    other split's entry."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    out = _run_bench(["--steps", "2", "--warmup", "1", "--batch", "16", "--global-batch", "16", "--cpu-sample", "0",
                      "--stream-sweeps", "0", "--latency-runs", "0", "--profile-steps", "1"], {})
    assert out["n_gpus"] == 1 and out["config"]["global_batch"] == 16
    share = out["weak"]["one_gpu_at_8gpu_share"]
    assert share["problems"] == 2 and share["value"] > 0 and share["ms_per_step"] > 0
