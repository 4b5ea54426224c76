"""The scenarios of tests/scenarios.py take the reference branches they are meant to take, in the
oracle (CPU): the GPU parity tests (test_gpu_branches.py) then compare the engine against these
same runs.  References: recentring src/laserMapping.cpp:446-614, degeneracy
src/laserOdometry.cpp:770-797 / src/laserMapping.cpp:927-954, NaN guard
src/laserOdometry.cpp:799-811, frameCount = skipFrameNum src/laserOdometry.cpp:407,885-891."""
import numpy as np

import scenarios


def test_grid_jumps_shift_every_axis(oc, sg):
    recs = scenarios.run_stream(oc.Oracle(oc.default_config(system_delay=1)), sg.stream_sweeps(34, 1),
                                jumps=scenarios.GRID_JUMPS)
    maps = [r for r in recs if "aft" in r]
    assert len(maps) >= len(scenarios.GRID_JUMPS)
    shifts = [r["mp_shifts"] for r in maps[:len(scenarios.GRID_JUMPS)]]
    # one slab per jump of 400 m / 140 m / 420 m, two for 150 m down, 16 for the 1100 m jump
    assert shifts[4] == 1 and shifts[6] == 1 and shifts[8] == 1 and shifts[10] == 2 and shifts[12] == 16, shifts
    assert sum(shifts) >= 40
    # the map survives the one-slab shifts: the frame after each jump matches against it again
    for k in (5, 7, 9, 11):
        assert maps[k]["mp_iters"] > 0, k
    # the 1100 m jump cleared the origin's cubes: no L-M on the way back
    assert maps[13]["mp_iters"] == 0


def test_ground_plane_is_degenerate(oc, sg):
    prev, cur = sg.single_problem(0)
    od, aft, st = oc.problem(scenarios.ground_only(prev), scenarios.ground_only(cur))
    assert st["od_iters"] > 0 and st["od_degenerate_steps"] == st["od_iters"]
    assert st["mp_iters"] > 0 and st["mp_degenerate_steps"] == st["mp_iters"]
    assert np.all(np.isfinite(od)) and np.all(np.isfinite(aft))


def test_coincident_corner_pair_trips_nan_guard(oc, sg):
    recs = scenarios.run_stream(oc.Oracle(oc.default_config(system_delay=1)), sg.stream_sweeps(8, 1),
                                mapping=False, inject_nan_at=4)
    hit = [r for r in recs if r["od_nan"]]
    assert len(hit) == 1 and hit[0]["k"] == 5
    assert hit[0]["od_nan"] == hit[0]["od_iters"] == 25   # rows accumulate (Q12): every step is NaN
    assert np.all(np.isfinite(hit[0]["pose"]))


def test_skip_frame_num_cadence(oc, sg):
    """frameCount starts at skipFrameNum: the first solved frame publishes the clouds"""
    sweeps = sg.stream_sweeps(12, 1)
    for skip in (0, 1, 2, 3):
        recs = scenarios.run_stream(oc.Oracle(oc.default_config(system_delay=1, skip_frame_num=skip)), sweeps,
                                    mapping=False, stats=False)
        solved = [r["pub"] for r in recs[1:]]
        expect = [7 if i % (skip + 1) == 0 else 1 for i in range(len(solved))]
        assert solved == expect, (skip, solved)


def test_q11_window_past_last_cloud(oc, sg):
    """Last clouds cut below the next sweep's sharp / flat counts: the L-M still runs (gates 10 /
    100) with forward windows that reach the ends of CornerLast / SurfLast (Q11, clamped at |Last|,
    src/laserOdometry.cpp:486, :598); tools/asan_suite.sh runs this under AddressSanitizer"""
    recs = scenarios.run_stream(oc.Oracle(oc.default_config(system_delay=1)), sg.stream_sweeps(12, 1),
                                truncate_last_at=(4, 7))
    by_k = {r["k"]: r for r in recs}
    for k in (4, 7):
        cut, nxt = by_k[k], by_k[k + 1]
        assert (cut["n_less_sharp"], cut["n_less_flat"]) == (14, 120)
        assert nxt["n_sharp"] > 14 and nxt["n_flat"] > 120
        assert nxt["od_iters"] > 0 and np.all(np.isfinite(nxt["pose"]))
