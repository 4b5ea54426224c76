"""loam_batch_feed: independent batches arriving over time through the step pipeline.

The pipeline's pre-runs (a step's scan registration + odometry seed enqueued during the previous
step) must take the fed sweeps, not the resident ones: every download after a feed sequence equals a
one-step run of the batch fed last, bit for bit (same kernels, same launch shapes)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _one_shot(loam, prevs, curs):
    e = loam.Engine()
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, st = e.batch_download()
    e.close()
    return od, aft, st


def _eq(got, want, what):
    np.testing.assert_array_equal(got[0], want[0], err_msg=what)
    np.testing.assert_array_equal(got[1], want[1], err_msg=what)
    for k in ("od_iters", "mp_iters", "n_raw", "n_sharp", "od_corner_last"):
        assert got[2][k] == want[2][k], (what, k)


@pytest.mark.parametrize("P", [128, 8], ids=["pipelined", "sequential"])
def test_feed_fresh_batches(loam, sg, P):
    A = sg.batch_problems(P, base_seed=1896)
    B = sg.batch_problems(P, base_seed=3000)
    ra, rb = _one_shot(loam, *A), _one_shot(loam, *B)
    assert not np.array_equal(ra[0], rb[0])
    e = loam.Engine()
    e.batch_upload(*A)
    pa, pb = e.prepare_batch(*A), e.prepare_batch(*B)
    # several steps in flight between downloads (each download drains the pipeline)
    for seq, want in (([pb], rb), ([pa, pb], rb), ([pb, pa, pb, pa], ra), ([pa, pa, pb], rb), ([pb, pb], rb)):
        for fb in seq:
            e.batch_feed(fb)
            e.batch_run()
        _eq(e.batch_download(), want, f"P={P} after {len(seq)} fed steps")
    # a run without a feed re-runs the sweeps resident in the set it reads
    e.batch_feed(pa)
    e.batch_run()
    e.batch_run()
    e.batch_feed(pa)
    e.batch_run()
    _eq(e.batch_download(), ra, "fed after an unfed run")
    e.close()


def test_feed_rejects_other_sizes(loam, sg):
    prevs, curs = sg.batch_problems(4, base_seed=1000)
    e = loam.Engine()
    with pytest.raises(loam.LoamError):
        e.batch_feed(prevs, curs)  # nothing uploaded
    e.batch_upload(prevs, curs)
    with pytest.raises(loam.LoamError):
        e.batch_feed(prevs[:3], curs[:3])
    e.close()
