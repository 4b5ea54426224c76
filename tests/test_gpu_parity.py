"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on identical inputs.

Tolerances: discrete outputs (ring order, feature selection, voxel membership) and point
coordinates are compared bit-exactly; the per-point `intensity` (ring + 0.1*relTime, from float
atan2: ocml on the GPU, glibc in the oracle) within 2e-6; poses within the north-star bound of
1e-4 m / 1e-4 rad (BASELINE.json)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4
INT_TOL = 2e-6


def _sr_both(loam, oc, raw, cfg_kw=None):
    cfg_kw = dict(cfg_kw or {})
    cfg_kw.setdefault("system_delay", 1)
    e = loam.Engine(loam.default_config(**cfg_kw))
    o = oc.Oracle(oc.default_config(**cfg_kw))
    assert e.scan_registration(raw)[0] == loam.LOAM_E_NOT_READY
    assert o.scan_registration(raw)[0] == loam.LOAM_E_NOT_READY
    rc, fg = e.scan_registration(raw)
    assert rc == 0
    rc, fo = o.scan_registration(raw)
    assert rc == 0
    return fg, fo


def _cmp_cloud(a, b, name):
    assert a.shape == b.shape, f"{name}: {a.shape} vs {b.shape}"
    np.testing.assert_array_equal(a[:, :3], b[:, :3], err_msg=name)
    if a.shape[0]:
        assert np.max(np.abs(a[:, 3] - b[:, 3])) <= INT_TOL, name


def test_sr_vlp16_single_sweep(loam, oc, sg):
    prev, cur = sg.single_problem(0)
    fg, fo = _sr_both(loam, oc, cur)
    for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
        _cmp_cloud(fg[k], fo[k], k)


def test_sr_hdl64(loam, oc, sg):
    prev, cur = sg.single_problem(2, lidar=sg.HDL64)
    kw = dict(n_rings=64, ring_model=loam.RING_LINEAR, max_points=160000)
    fg, fo = _sr_both(loam, oc, cur, kw)
    for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
        _cmp_cloud(fg[k], fo[k], k)


def test_sr_random_scenes(loam, oc, sg):
    prevs, curs = sg.batch_problems(4, base_seed=1000)
    for raw in prevs + curs:
        fg, fo = _sr_both(loam, oc, raw)
        for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
            _cmp_cloud(fg[k], fo[k], k)


def test_sr_nan_and_ragged(loam, oc, sg):
    _, cur = sg.single_problem(0)
    raw = cur.copy()
    raw[::97, 0] = np.nan          # non-finite returns are filtered (removeNaNFromPointCloud)
    raw = raw[: 20011]             # ragged length, partial sweep
    fg, fo = _sr_both(loam, oc, raw)
    for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
        _cmp_cloud(fg[k], fo[k], k)


def test_sr_empty_ring(loam, oc, sg):
    # a missing ring leaves its predecessor's end index at 0 (Q5): the ring spans overlap and the
    # rings are selected in order by one workgroup (the dependent-ring path)
    _, cur = sg.single_problem(0)
    elev = np.degrees(np.arctan2(cur[:, 2], np.hypot(cur[:, 0], cur[:, 1])))
    raw = cur[np.abs(elev - 3.0) > 0.5]
    assert raw.shape[0] < cur.shape[0]
    fg, fo = _sr_both(loam, oc, raw)
    for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
        _cmp_cloud(fg[k], fo[k], k)


def test_sr_long_rings(loam, oc, sg):
    # two sweeps in one message: 3600 points per ring, beyond the 2048-point fast selection kernel
    prev, cur = sg.single_problem(0)
    raw = np.concatenate([prev, cur])
    fg, fo = _sr_both(loam, oc, raw, dict(max_points=80000))
    for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
        _cmp_cloud(fg[k], fo[k], k)


def test_sr_batch_selection_routes(loam, oc, sg):
    """A batch whose sweeps take every selection route at once, more of them than the fallback
    kernels' workgroup rows (sr.hip kSelListGrid): problems with an empty ring (dependent rings,
    k_sr_select<4096, 1>), two sweeps per message (3600-point rings, the same kernel) and both
    (a predecessor spanning two long rings, past 4096 points: k_sr_select<16, 2>), between plain
    ones (k_sr_pick / k_sr_ringvg).  Every problem's poses against the oracle."""
    P = 48
    prevs, curs = sg.batch_problems(P + 1, base_seed=3000)

    def drop_ring(a):
        elev = np.degrees(np.arctan2(a[:, 2], np.hypot(a[:, 0], a[:, 1])))
        return a[np.abs(elev - 3.0) > 0.5]

    bp, bc = [], []
    for i in range(P):
        p, c = prevs[i], curs[i]
        if i % 4 in (1, 3):  # two sweeps per message
            p, c = np.concatenate([prevs[i + 1], p]), np.concatenate([p, c])
        if i % 4 in (0, 3):
            p, c = drop_ring(p), drop_ring(c)
        bp.append(p)
        bc.append(c)
    kw = dict(max_points=80000)
    e = loam.Engine(loam.default_config(**kw))
    e.batch_upload(bp, bc)
    e.batch_run()
    od, aft, _ = e.batch_download()
    e.close()
    ocfg = oc.default_config(**kw)
    for i in range(P):
        od_o, aft_o, _ = oc.problem(bp[i], bc[i], ocfg)
        assert max(np.abs(od[i] - od_o).max(), np.abs(aft[i] - aft_o).max()) <= POSE_TOL, i


@pytest.mark.parametrize("model", ["vlp16", "linear64"])
def test_sr_ring_boundaries(loam, oc, sg, model):
    """Every third point moved to within 1e-7..3e-3 degrees of a ring boundary: the engine's float
    ring ID defers to the double evaluation there (sr.hip ring_of), the oracle always uses double."""
    if model == "vlp16":
        _, raw = sg.single_problem(0)
        kw = {}
        bounds = np.arange(-16.0, 17.0, 2.0)  # round((angle + 15) / 2) steps at even degrees
    else:
        _, raw = sg.single_problem(2, lidar=sg.HDL64)
        kw = dict(n_rings=64, ring_model=loam.RING_LINEAR, max_points=160000)
        c = loam.default_config(**kw)
        step = (c.ring_hi_deg - c.ring_lo_deg) / 63
        bounds = c.ring_lo_deg + (np.arange(64) + 0.5) * step
    raw = raw.copy()
    rng = np.random.default_rng(7)
    sel = np.arange(0, raw.shape[0], 3)
    h = np.hypot(raw[sel, 0], raw[sel, 1]).astype(np.float64)
    ang = np.degrees(np.arctan2(raw[sel, 2], h))
    near = bounds[np.abs(ang[:, None] - bounds[None, :]).argmin(axis=1)]
    off = rng.choice([-1.0, 1.0], sel.size) * 10.0 ** rng.uniform(-7, np.log10(3e-3), sel.size)
    raw[sel, 2] = (np.tan(np.radians(near + off)) * h).astype(np.float32)
    fg, fo = _sr_both(loam, oc, raw, kw)
    for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
        _cmp_cloud(fg[k], fo[k], k)


def test_sr_stride32(loam, oc, sg):
    _, cur = sg.single_problem(0)
    raw = np.zeros((cur.shape[0], 8), np.float32)   # PointXYZI-like 32-byte records
    raw[:, :4] = cur
    fg, fo = _sr_both(loam, oc, raw)
    _cmp_cloud(fg["less_flat"], fo["less_flat"], "less_flat")


def _stream(impl, sweeps, mapping=False):
    poses, maps = [], []
    for k, sw in enumerate(sweeps):
        rc, f = impl.scan_registration(sw, stamp=0.1 * k)
        if rc != 0:
            continue
        pub, pose, cl, sl, full = impl.odometry(f, stamp=0.1 * k)
        if pub & 1:
            poses.append(pose)
        if mapping and pub == 7:
            aft, bef, reg = impl.mapping(pose, cl, sl, full)
            maps.append((aft, bef, impl.mapping_surround()))
    return np.array(poses), maps


def test_odometry_stream_parity(loam, oc, sg):
    sweeps = sg.stream_sweeps(30, 1)
    cfg = dict(system_delay=2)
    pg, _ = _stream(loam.Engine(loam.default_config(**cfg)), sweeps)
    po, _ = _stream(oc.Oracle(oc.default_config(**cfg)), sweeps)
    assert pg.shape == po.shape and pg.shape[0] >= 20
    err = np.abs(pg - po).max(axis=1)
    assert err.max() <= POSE_TOL, err


def test_batch_odometry_parity(loam, oc, sg):
    prevs, curs = sg.batch_problems(8, base_seed=1000)
    e = loam.Engine()
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, st = e.batch_download()
    for i in range(len(prevs)):
        od_o, aft_o, st_o = oc.problem(prevs[i], curs[i])
        assert np.abs(od[i] - od_o).max() <= POSE_TOL, (i, od[i], od_o)


def test_batch_single_problem_config2(loam, oc, sg):
    prev, cur = sg.single_problem(0)
    e = loam.Engine()
    e.batch_upload([prev], [cur])
    e.batch_run()
    od, aft, st = e.batch_download()
    od_o, aft_o, st_o = oc.problem(prev, cur)
    assert np.abs(od[0] - od_o).max() <= POSE_TOL
    assert st["od_iters"] == st_o["od_iters"]


def test_mapping_stream_parity(loam, oc, sg):
    sweeps = sg.stream_sweeps(30, 1)
    cfg = dict(system_delay=2)
    pg, mg = _stream(loam.Engine(loam.default_config(**cfg)), sweeps, mapping=True)
    po, mo = _stream(oc.Oracle(oc.default_config(**cfg)), sweeps, mapping=True)
    assert len(mg) == len(mo) >= 10
    nsur = 0
    for k, ((ag, bg, sg_), (ao, bo, so)) in enumerate(zip(mg, mo)):
        assert np.abs(ag - ao).max() <= POSE_TOL
        assert np.abs(bg - bo).max() <= POSE_TOL
        # /laser_cloud_surround: 1st mapping frame, then every 5th (laserMapping.cpp:1038-1058)
        assert (sg_ is not None) == (so is not None) == (k % 5 == 0), k
        if so is not None:
            assert sg_.shape == so.shape and so.shape[0] > 100
            assert np.array_equal(sg_, so), np.abs(sg_ - so).max()
            nsur += 1
    assert nsur >= 2


def test_golden_config3_stream(loam, sg):
    import json, os, hashlib
    G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))
    sweeps = sg.stream_sweeps(30, 1)
    e = loam.Engine(loam.default_config(system_delay=2))
    traj = []
    for k, sw in enumerate(sweeps):
        rc, f = e.scan_registration(sw)
        if rc:
            continue
        pub, pose, cl, sl, full = e.odometry(f)
        rec = {"pub": pub, "od": pose}
        if pub == 7:
            a, b, reg = e.mapping(pose, cl, sl, full)
            rec.update(aft=a, bef=b, reg=hashlib.sha256(np.ascontiguousarray(reg, np.float32).tobytes()).hexdigest())
            sur = e.mapping_surround()
            rec["sur"] = None if sur is None else hashlib.sha256(np.ascontiguousarray(sur, np.float32).tobytes()).hexdigest()
        traj.append(rec)
    assert len(traj) == len(G["config3_first30"])
    for r, g in zip(traj, G["config3_first30"]):
        assert r["pub"] == g["pub"]
        if g["od_sum"] is not None:
            assert np.abs(r["od"] - np.float32(g["od_sum"])).max() <= POSE_TOL
        if "aft" in g:
            assert np.abs(r["aft"] - np.float32(g["aft"])).max() <= POSE_TOL
            assert r["reg"] == g["registered_sha256"]   # /velodyne_cloud_registered, bit-exact
            assert r["sur"] == g.get("surround_sha256")


def test_golden_config4(loam, sg):
    import json, os
    G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))
    prevs, curs = sg.batch_problems(8, base_seed=1000)
    e = loam.Engine()
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, st = e.batch_download()
    for i in range(8):
        assert np.abs(od[i] - np.float32(G["config4_first8"][i]["od_sum"])).max() <= POSE_TOL
        assert np.abs(aft[i] - np.float32(G["config4_first8"][i]["aft"])).max() <= POSE_TOL


def test_batch_mapping_parity_64(loam, oc, sg):
    prevs, curs = sg.batch_problems(64, base_seed=1100)
    e = loam.Engine()
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, st = e.batch_download()
    errs = []
    for i in range(64):
        od_o, aft_o, _ = oc.problem(prevs[i], curs[i])
        errs.append(max(np.abs(od[i] - od_o).max(), np.abs(aft[i] - aft_o).max()))
    assert max(errs) <= POSE_TOL, errs
    # the repeated run of the same batch is deterministic
    e.batch_run()
    od2, aft2, _ = e.batch_download()
    np.testing.assert_array_equal(od, od2)
    np.testing.assert_array_equal(aft, aft2)


def test_batch_sparse_map_parity(loam, oc, sg):
    """Maps built from a thinned previous sweep (every 4th return): many 5-NN searches end with the
    fifth neighbour at >= 1 m (rejected, :719 / :826) — lists left holding copies of the bound B,
    seeds withheld from the next iteration (q_nn distinct flag) — and the poses must still follow
    the oracle, the same on a repeated run."""
    prevs, curs = sg.batch_problems(16, base_seed=1400)
    prevs = [p[::4].copy() for p in prevs]
    e = loam.Engine()
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, _ = e.batch_download()
    for i in range(16):
        od_o, aft_o, _ = oc.problem(prevs[i], curs[i])
        assert max(np.abs(od[i] - od_o).max(), np.abs(aft[i] - aft_o).max()) <= POSE_TOL, i
    e.batch_run()
    od2, aft2, _ = e.batch_download()
    np.testing.assert_array_equal(od, od2)
    np.testing.assert_array_equal(aft, aft2)


def _push_out(raw, rng_m=250.0, az_deg=(0.0, 12.0)):
    """top-ring returns within an azimuth block moved out to rng_m metres along their rays"""
    raw = raw.copy()
    h = np.hypot(raw[:, 0], raw[:, 1])
    el = np.degrees(np.arctan2(raw[:, 2], h))
    az = np.degrees(np.arctan2(raw[:, 1], raw[:, 0])) % 360.0
    sel = (el > 14.0) & (az >= az_deg[0]) & (az < az_deg[1])
    r = np.linalg.norm(raw[sel, :3], axis=1, keepdims=True)
    raw[sel, :3] = (raw[sel, :3] / r * rng_m).astype(np.float32)
    return raw, int(sel.sum())


def test_batch_stack_keys_beyond_24_bits(loam, oc, sg):
    """Batch mapping with stacks whose 0.4 m VoxelGrid spans more than 2^24 voxels (far returns on
    the top ring): the VoxelGrid cascade's radix passes must cover every bit the keys span."""
    prevs, curs = sg.batch_problems(8, base_seed=1300)
    for i in (0, 3, 6):
        prevs[i], n0 = _push_out(prevs[i])
        curs[i], n1 = _push_out(curs[i])
        assert n0 > 20 and n1 > 20
    o = oc.Oracle(oc.default_config(system_delay=1))
    o.scan_registration(curs[0])
    _, f = o.scan_registration(curs[0])
    lf = f["less_flat"][:, :3]
    ext = np.floor(lf.max(axis=0) / 0.4) - np.floor(lf.min(axis=0) / 0.4) + 1
    assert np.prod(ext) > 2 ** 25, ext
    e = loam.Engine()
    e.batch_upload(prevs, curs)
    e.batch_run()
    od, aft, _ = e.batch_download()
    for i in range(8):
        od_o, aft_o, _ = oc.problem(prevs[i], curs[i])
        assert max(np.abs(od[i] - od_o).max(), np.abs(aft[i] - aft_o).max()) <= POSE_TOL, i


def test_hdl64_problem_config5(loam, oc, sg):
    prev, cur = sg.single_problem(2, lidar=sg.HDL64)
    kw = dict(n_rings=64, ring_model=loam.RING_LINEAR, max_points=160000)
    e = loam.Engine(loam.default_config(**kw))
    e.batch_upload([prev], [cur])
    e.batch_run()
    od, aft, st = e.batch_download()
    od_o, aft_o, _ = oc.problem(prev, cur, oc.default_config(**kw))
    assert np.abs(od[0] - od_o).max() <= POSE_TOL
    assert np.abs(aft[0] - aft_o).max() <= POSE_TOL


def test_capacity_and_empty_errors(loam, sg):
    e = loam.Engine(loam.default_config(system_delay=0, max_points=20000))
    _, cur = sg.single_problem(0)
    e.scan_registration(cur[:100])                      # consumed by systemDelay
    with pytest.raises(loam.LoamError) as ei:
        e.scan_registration(cur)                        # 28800 > max_points
    assert ei.value.code == loam.LOAM_E_CAPACITY
    nan = np.full((50, 4), np.nan, np.float32)
    with pytest.raises(loam.LoamError) as ei:
        e.scan_registration(nan)
    assert ei.value.code == loam.LOAM_E_INVAL


def test_batch_empty_and_tiny_sweeps(loam, oc, sg):
    """a batch with a sweep of no finite point fails as the node call does (LOAM_E_INVAL at the
    download) and leaves the context usable; a batch with a 300-point sweep (most rings empty, few or
    no features) runs through every batch kernel and equals the oracle"""
    prevs, curs = sg.batch_problems(8, base_seed=4100)
    bad = list(curs)
    bad[2] = np.full((100, 4), np.nan, np.float32)
    e = loam.Engine()
    e.batch_upload(prevs, bad)
    e.batch_run()
    with pytest.raises(loam.LoamError) as ei:
        e.batch_download()
    assert ei.value.code == loam.LOAM_E_INVAL
    tiny = list(prevs)
    tiny[5] = prevs[5][:300]
    e.batch_upload(tiny, curs)
    e.batch_run()
    od, aft, _ = e.batch_download()
    e.close()
    assert np.all(np.isfinite(od)) and np.all(np.isfinite(aft))
    for i in (0, 5, 7):
        od_o, aft_o, _ = oc.problem(tiny[i], curs[i])
        assert max(np.abs(od[i] - od_o).max(), np.abs(aft[i] - aft_o).max()) <= POSE_TOL, i


def test_maintenance_chain(loam, oc, sg):
    prev, cur = sg.single_problem(0)
    e = loam.Engine()
    e.batch_upload([prev], [cur])
    e.batch_run()
    od, aft, st = e.batch_download()
    np.testing.assert_array_equal(loam.maintenance(od[0], od[0], aft[0]), oc.maintenance(od[0], od[0], aft[0]))


def _stream_imu(impl, sweeps, imus, t0, with_feats=False):
    """config-3 style stream with /imu/data delivered up to each sweep's end before the sweep"""
    j, poses, maps, feats = 0, [], [], []
    for k, sw in enumerate(sweeps):
        while j < len(imus) and imus[j][0] <= t0 + 0.1 * (k + 1):
            impl.imu(*imus[j])
            j += 1
        rc, f = impl.scan_registration(sw, stamp=t0 + 0.1 * k)
        if rc != 0:
            continue
        if with_feats:
            feats.append(f)
        pub, pose, cl, sl, full = impl.odometry(f, stamp=t0 + 0.1 * k)
        if pub & 1:
            poses.append(pose)
        if pub == 7:
            aft, bef, reg = impl.mapping(pose, cl, sl, full, stamp=t0 + 0.1 * k)
            maps.append((aft, bef))
    return np.array(poses), maps, feats


def test_imu_stream_parity(loam, oc, sg):
    # the IMU path: per-point de-skew with the interpolated IMU state and /imu_trans
    # (scanRegistration), the IMU prior / TransformToEnd / PluginIMURotation terms (odometry), the
    # roll / pitch blend of transformUpdate (mapping)
    t0 = 0.0
    sweeps = sg.stream_sweeps(24, 1, t0=t0)
    imus = sg.imu_stream(t0 - 0.5, t0 + 2.5, seed=1)
    cfg = dict(system_delay=2)
    pg, mg, fg = _stream_imu(loam.Engine(loam.default_config(**cfg)), sweeps, imus, t0, with_feats=True)
    po, mo, fo = _stream_imu(oc.Oracle(oc.default_config(**cfg)), sweeps, imus, t0, with_feats=True)
    assert len(fg) == len(fo) >= 20
    for a, b in zip(fg, fo):
        np.testing.assert_array_equal(a["imu_trans"], b["imu_trans"])
        assert np.abs(a["imu_trans"]).max() > 0
        for k in ("full", "sharp", "less_sharp", "flat", "less_flat"):
            _cmp_cloud(a[k], b[k], k)
    assert len(pg) == len(po) and np.abs(pg - po).max() <= POSE_TOL
    assert len(mg) == len(mo) >= 8
    for (ag, bg), (ao, bo) in zip(mg, mo):
        assert np.abs(ag - ao).max() <= POSE_TOL
        assert np.abs(bg - bo).max() <= POSE_TOL


def test_imu_errors(loam, sg):
    e = loam.Engine()
    e.imu(1.0, (0, 0, 0, 1), (0, 0, 9.81))
    with pytest.raises(loam.LoamError):
        e.imu(0.5, (0, 0, 0, 1), (0, 0, 9.81))   # stamps must be non-decreasing


def test_golden_config3_imu(loam, sg):
    from test_golden import _imu_stream, check_imu_traj
    check_imu_traj(_imu_stream(loam.Engine(loam.default_config(system_delay=2)), sg), tol=POSE_TOL)
