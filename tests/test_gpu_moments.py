"""The odometry's Q12 row re-evaluation as per-query moments (tuning od_moments_min)
against the oracle on EVERY problem of the benched batches.

The reference re-evaluates every stored row's Jacobian each L-M iteration with float J entries
(src/laserOdometry.cpp:697-764, Q12).  The moments form sums the same rows as E_q M_q E_qᵀ in fp64,
so it is not bit-identical: the bar is the north star's 1e-4 m / 1e-4 rad on the odometry and the
mapping pose of every problem.  The bit-exact form (od_moments_min above the batch size) is checked
against the same oracle runs bit for bit, poses and per-problem L-M iteration counts, so both forms
are pinned on all 1024 config-4 problems and all 64 config-5 problems.

Every moments error is attributed.  The fp64 moments round the odometry's normal equations
differently from the reference's float J entries: a ~1e-7 relative perturbation of each L-M step,
which leaves the odometry within a few float ulps of the reference (<= ATTRIB).  A larger error
has one of two causes, and the test names it for every such problem:
  * a convergence test flipped (ΔR < 0.1° and ΔT < 0.1 cm odometry, 0.05 / 0.05 mapping,
    src/laserOdometry.cpp:824, src/laserMapping.cpp:972): the problem's iteration count differs;
  * the reference's mapping itself moves that far for an odometry input a few ulps away (a 5-NN /
    acceptance decision at a threshold in :714-877, on a problem whose mapping L-M does not
    converge): replaying the oracle with the engine's solved odometry transform
    (oracle_problem_with_od) gives the engine's mapping pose to within ATTRIB.
The test prints the error histogram and every problem above ATTRIB with its cause.  The oracle runs on a thread pool (ctypes releases the GIL; the oracle keeps no
global state)."""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north star: output transforms within 1e-4 m / 1e-4 rad
ATTRIB = 1e-6  # the largest error the moments' rounding alone is allowed without a convergence flip
DENSE = dict(n_rings=64, max_points=160000, od_max_iter=100, mp_max_iter=20)


def _oracle_all(oc, prevs, curs, ocfg=None):
    n = min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(n) as ex:
        outs = list(ex.map(lambda pc: oc.problem(pc[0], pc[1], ocfg), zip(prevs, curs)))
    od = np.array([o[0] for o in outs])
    aft = np.array([o[1] for o in outs])
    od_it = np.array([o[2]["od_iters"] for o in outs])
    mp_it = np.array([o[2]["mp_iters"] for o in outs])
    return od, aft, od_it, mp_it


def _run(loam, prevs, curs, cfg, **tune):
    e = loam.Engine(cfg) if cfg is not None else loam.Engine()
    e.set_tuning(**tune)
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, st = e.batch_download()
    od_it, mp_it, tr = e.batch_lm_info()
    e.close()
    return od, aft, st, od_it, mp_it, tr


def _check(loam, oc, prevs, curs, cfg, ocfg, oracle):
    od_o, aft_o, od_it_o, mp_it_o = oracle
    exact = _run(loam, prevs, curs, cfg, od_moments_min=1 << 30)
    mom = _run(loam, prevs, curs, cfg, od_moments_min=1)
    # the reference's row re-evaluation: bit-exact on every problem, every convergence decision equal
    np.testing.assert_array_equal(exact[0], od_o)
    np.testing.assert_array_equal(exact[1], aft_o)
    np.testing.assert_array_equal(exact[3], od_it_o)
    np.testing.assert_array_equal(exact[4], mp_it_o)
    # the moments: every problem within the north star, every error above ATTRIB explained by a flip
    e_od = np.abs(mom[0] - od_o).max(axis=1)
    e_mp = np.abs(mom[1] - aft_o).max(axis=1)
    err = np.maximum(e_od, e_mp)
    flip_od = mom[3] != od_it_o
    flip_mp = mom[4] != mp_it_o
    edges = [0.0, 1e-9, 1e-8, 1e-7, 1e-6, 1e-5, TOL, np.inf]
    hist = {f"<= {edges[i + 1]:.0e}" if i else "== 0": int(np.sum((err > edges[i]) & (err <= edges[i + 1])) if i
                                                        else np.sum(err == 0))
            for i in range(len(edges) - 1)}
    print(f"moments: {len(prevs)} problems, max |d odometry| {e_od.max():.3g}, max |d mapping| {e_mp.max():.3g}; "
          f"error histogram {hist}; odometry iterations {int(mom[3].sum())} vs oracle {int(od_it_o.sum())}, "
          f"mapping {int(mom[4].sum())} vs {int(mp_it_o.sum())}")
    assert e_od.max() <= ATTRIB or np.all(flip_od[e_od > ATTRIB]), "odometry error without a flip"
    unexplained = []
    for i in np.flatnonzero(flip_od | flip_mp | (err > ATTRIB)):
        cause = "odometry convergence flip" if flip_od[i] else "mapping convergence flip" if flip_mp[i] else None
        if cause is None:  # the reference's mapping for the engine's odometry result
            _, aft_r, _ = oc.problem_with_od(prevs[i], curs[i], mom[5][i], ocfg)
            d = float(np.abs(mom[1][i] - aft_r).max())
            cause = f"reference mapping for this odometry result within {d:.2g} of the engine's"
            if d > ATTRIB:
                unexplained.append(int(i))
        print(f"  problem {i}: |d odometry| {e_od[i]:.3g} |d mapping| {e_mp[i]:.3g}; odometry iterations "
              f"{mom[3][i]} (oracle {od_it_o[i]}), mapping {mom[4][i]} (oracle {mp_it_o[i]}): {cause}")
    assert err.max() <= TOL, int(np.argmax(err))
    assert not unexplained, f"errors above {ATTRIB} with no identified cause: {unexplained}"
    return mom


def test_moments_config4_all_1024(loam, oc, sg):
    P = 1024
    prevs, curs = sg.batch_problems(P, base_seed=1000)
    _check(loam, oc, prevs, curs, None, None, _oracle_all(oc, prevs, curs))


def test_moments_config5_all_64(loam, oc, sg):
    P = 64
    prevs, curs = sg.batch_problems(P, base_seed=5000, lidar=sg.HDL64)
    cfg = loam.default_config(ring_model=loam.RING_LINEAR, **DENSE)
    ocfg = oc.default_config(ring_model=1, **DENSE)
    _check(loam, oc, prevs, curs, cfg, ocfg, _oracle_all(oc, prevs, curs, ocfg))


def test_moments_8gpu_share_fused(loam, oc, sg):
    """the share (P = 128): the moments in the fused rows kernel (step in the last workgroup) and
    through the step pipeline (three steps), against the oracle"""
    P, r = 128, 7
    prevs, curs = sg.batch_problems(P, base_seed=1000 + r * P)
    od_o, aft_o, _, _ = _oracle_all(oc, prevs, curs)
    e = loam.Engine()
    e.set_tuning(od_moments_min=1, step_pipe=1)
    e.batch_upload(prevs, curs)
    for _ in range(3):
        e.batch_run()
    od, aft, _ = e.batch_download()
    e.close()
    assert np.abs(od - od_o).max() <= TOL and np.abs(aft - aft_o).max() <= TOL


@pytest.mark.parametrize("tune", [{"od_fused_max": 0}, {"step_pipe": 0, "sr_ahead": 0}, {"graph": 1}],
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
