"""The odometry's Q12 row re-evaluation as per-query moments (tuning od_moments_min)
against the oracle on EVERY problem of the benched batches.

The reference re-evaluates every stored row's Jacobian each L-M iteration with float J entries
(src/laserOdometry.cpp:697-764, Q12).  The moments form sums the same rows as E_q M_q E_qᵀ in fp64,
so it is not bit-identical: the bar is the north star's 1e-4 m / 1e-4 rad on the odometry and the
mapping pose of every problem.  The bit-exact form (the default at these sizes unless the default
changes) is checked against the same oracle runs bit for bit, so both forms are pinned on all
1024 config-4 problems and all 64 config-5 problems.  The oracle runs on a thread pool (ctypes
releases the GIL; the oracle keeps no global state)."""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north star: output transforms within 1e-4 m / 1e-4 rad
DENSE = dict(n_rings=64, max_points=160000, od_max_iter=100, mp_max_iter=20)


def _oracle_all(oc, prevs, curs, ocfg=None):
    n = min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(n) as ex:
        outs = list(ex.map(lambda pc: oc.problem(pc[0], pc[1], ocfg), zip(prevs, curs)))
    od = np.array([o[0] for o in outs])
    aft = np.array([o[1] for o in outs])
    iters = sum(o[2]["od_iters"] for o in outs)
    return od, aft, iters


def _run(loam, prevs, curs, cfg, **tune):
    e = loam.Engine(cfg) if cfg is not None else loam.Engine()
    e.set_tuning(**tune)
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, st = e.batch_download()
    e.close()
    return od, aft, st


def _check(loam, prevs, curs, cfg, oracle):
    od_o, aft_o, iters_o = oracle
    exact = _run(loam, prevs, curs, cfg, od_moments_min=1 << 30)
    mom = _run(loam, prevs, curs, cfg, od_moments_min=1)
    # the reference's row re-evaluation: bit-exact on every problem
    np.testing.assert_array_equal(exact[0], od_o)
    np.testing.assert_array_equal(exact[1], aft_o)
    assert exact[2]["od_iters"] == iters_o
    # the moments: every problem within the north star
    e_od = np.abs(mom[0] - od_o).max(axis=1)
    e_mp = np.abs(mom[1] - aft_o).max(axis=1)
    worst = int(np.argmax(np.maximum(e_od, e_mp)))
    print(f"moments: {len(prevs)} problems, max |d odometry| {e_od.max():.3g}, max |d mapping| "
          f"{e_mp.max():.3g} (problem {worst}), bit-identical {int(np.sum((e_od == 0) & (e_mp == 0)))}, "
          f"odometry iterations {mom[2]['od_iters']} vs oracle {iters_o}")
    assert e_od.max() <= TOL and e_mp.max() <= TOL, worst
    return mom


def test_moments_config4_all_1024(loam, oc, sg):
    P = 1024
    prevs, curs = sg.batch_problems(P, base_seed=1000)
    _check(loam, prevs, curs, None, _oracle_all(oc, prevs, curs))


def test_moments_config5_all_64(loam, oc, sg):
    P = 64
    prevs, curs = sg.batch_problems(P, base_seed=5000, lidar=sg.HDL64)
    cfg = loam.default_config(ring_model=loam.RING_LINEAR, **DENSE)
    _check(loam, prevs, curs, cfg, _oracle_all(oc, prevs, curs, oc.default_config(ring_model=1, **DENSE)))


@pytest.mark.parametrize("P,seed,dense", [(128, 1896, False), (64, 5000, True)], ids=["share128", "config5"])
def test_moments_round_kernel(loam, oc, sg, P, seed, dense):
    """k_od_lm_mom (an association round's five iterations in one workgroup per problem, the rows as
    moments; tuning od_lm_mom_max) at the 8-GPU share and on config 5's 2304-query HDL-64E problems
    (144 KB of LDS per workgroup): every problem within the north star of the oracle"""
    kw = dict(lidar=sg.HDL64) if dense else {}
    prevs, curs = sg.batch_problems(P, base_seed=seed, **kw)
    cfg = loam.default_config(ring_model=loam.RING_LINEAR, **DENSE) if dense else None
    ocfg = oc.default_config(ring_model=1, **DENSE) if dense else None
    od_o, aft_o, iters_o = _oracle_all(oc, prevs, curs, ocfg)
    od, aft, st = _run(loam, prevs, curs, cfg, od_lm_mom_max=1 << 20)
    e_od, e_mp = np.abs(od - od_o).max(), np.abs(aft - aft_o).max()
    print(f"k_od_lm_mom P={P}: max |d odometry| {e_od:.3g}, |d mapping| {e_mp:.3g}, "
          f"iterations {st['od_iters']} vs {iters_o}")
    assert e_od <= TOL and e_mp <= TOL


def test_moments_8gpu_share_fused(loam, oc, sg):
    """the share (P = 128): the moments in the fused rows kernel (step in the last workgroup) and
    through the step pipeline (three steps), against the oracle"""
    P, r = 128, 7
    prevs, curs = sg.batch_problems(P, base_seed=1000 + r * P)
    od_o, aft_o, _ = _oracle_all(oc, prevs, curs)
    e = loam.Engine()
    e.set_tuning(od_moments_min=1, step_pipe=1)
    e.batch_upload(prevs, curs)
    for _ in range(3):
        e.batch_run()
    od, aft, _ = e.batch_download()
    e.close()
    assert np.abs(od - od_o).max() <= TOL and np.abs(aft - aft_o).max() <= TOL


@pytest.mark.parametrize("tune", [{"od_fused_max": 0}, {"step_pipe": 0, "sr_ahead": 0}, {"graph": 1},
                                  {"od_rows_deep_max": 128}],
                         ids=lambda t: ",".join(f"{k}={v}" for k, v in t.items()))
def test_moments_launch_choices_at_8gpu_share(loam, sg, tune):
    """the moments' launch choices compute the same sums in the same order: the fused rows kernel
    (step in the last workgroup) and k_od_rows + k_od_step, sequential and pipelined steps, a graph
    replay give the default's poses bit for bit (the moments run at P >= od_moments_min = 64)"""
    P, r = 128, 7
    prevs, curs = sg.batch_problems(P, base_seed=1000 + r * P)

    def run(**t):
        e = loam.Engine()
        assert e.get_tuning("od_moments_min") <= P
        e.set_tuning(**t)
        e.batch_upload(prevs, curs)
        for _ in range(3):
            e.batch_run()
        out = e.batch_download()
        e.close()
        return out

    od0, aft0, st0 = run()
    od, aft, st = run(**tune)
    np.testing.assert_array_equal(od, od0)
    np.testing.assert_array_equal(aft, aft0)
    assert st["od_iters"] == st0["od_iters"] and st["mp_iters"] == st0["mp_iters"]
