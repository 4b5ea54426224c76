"""Known-answer checks of the oracle's third-party restatements (PCL KdTreeFLANN / VoxelGrid,
OpenCV solve / eigen / inv, tf) against independent numpy computations.  The reference's own
tests hold no fixtures for these, so this is how the oracle is pinned."""
import ctypes

import numpy as np
import pytest


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


def test_knn_exact_with_index_tiebreak(oc):
    rng = np.random.default_rng(1)
    pts = _f32(np.round(rng.uniform(-5, 5, (3000, 4)), 1))   # coarse grid -> many equal distances
    q = _f32(np.round(rng.uniform(-5, 5, (400, 4)), 1))
    k = 5
    idx = np.zeros((400, k), np.int32)
    d = np.zeros((400, k), np.float32)
    oc.lib().oracle_knn(pts.ctypes.data, 3000, q.ctypes.data, 400, k, idx.ctypes.data, d.ctypes.data)
    for i in range(400):
        dd = ((pts[:, 0] - q[i, 0]) ** 2 + (pts[:, 1] - q[i, 1]) ** 2) + (pts[:, 2] - q[i, 2]) ** 2
        dd = dd.astype(np.float32)
        order = np.lexsort((np.arange(3000), dd))[:k]
        np.testing.assert_array_equal(idx[i], order)
        np.testing.assert_array_equal(d[i], dd[order])


def pcl_voxel_grid(pts, leaf):
    """independent numpy statement of pcl::VoxelGrid (PCL 1.7.1 applyFilter, all fields)"""
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = pts[:, :3].min(0), pts[:, :3].max(0)
    dxyz = ((mx - mn) * inv).astype(np.int64) + 1
    if int(np.prod(dxyz)) > 2 ** 31 - 1:
        return pts.copy()
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(mx * inv).astype(np.int64)
    div = maxb - minb + 1
    ijk = (np.floor(pts[:, :3] * inv) - minb.astype(np.float32)).astype(np.int64)
    key = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]).astype(np.uint32)
    order = np.lexsort((np.arange(len(pts)), key))
    out = []
    i = 0
    while i < len(order):
        j = i
        s = np.zeros(4, np.float32)
        while j < len(order) and key[order[j]] == key[order[i]]:
            s = (s + pts[order[j]]).astype(np.float32)
            j += 1
        out.append(s / np.float32(j - i))
        i = j
    return np.array(out, np.float32)


@pytest.mark.parametrize("leaf", [0.2, 0.4])
def test_voxel_grid_matches_pcl_statement(oc, leaf):
    rng = np.random.default_rng(2)
    pts = _f32(np.concatenate([rng.uniform(-20, 20, (5000, 3)), rng.uniform(0, 16, (5000, 1))], 1))
    out = np.zeros((5000, 4), np.float32)
    n = oc.lib().oracle_voxel_grid(pts.ctypes.data, 5000, leaf, out.ctypes.data, 5000)
    ref = pcl_voxel_grid(pts, leaf)
    assert n == len(ref)
    np.testing.assert_array_equal(out[:n], ref)


def test_voxel_grid_leaf_too_small_passthrough(oc):
    pts = _f32([[0, 0, 0, 1], [1e6, 1e6, 1e6, 2], [5, 5, 5, 3]])
    out = np.zeros((3, 4), np.float32)
    n = oc.lib().oracle_voxel_grid(pts.ctypes.data, 3, 0.2, out.ctypes.data, 3)
    assert n == 3
    np.testing.assert_array_equal(out, pts)


def test_qr_solve_square_and_least_squares(oc):
    rng = np.random.default_rng(3)
    for m, n in ((6, 6), (5, 3)):
        for _ in range(50):
            A = _f32(rng.normal(size=(m, n)))
            if m == n:
                A = _f32(A @ A.T + np.eye(n) * 2)
            b = _f32(rng.normal(size=m))
            x = np.zeros(n, np.float32)
            ok = oc.lib().oracle_qr_solve(A.ctypes.data, b.ctypes.data, m, n, x.ctypes.data)
            assert ok == 1
            ref = np.linalg.lstsq(A.astype(np.float64), b.astype(np.float64), rcond=None)[0]
            assert np.abs(x - ref).max() <= 1e-4 * max(1.0, np.abs(ref).max())


def test_qr_solve_rank_deficient(oc):
    # a vanishing R diagonal (< 10*FLT_EPSILON) makes cv::solve fail and output zeros
    rng = np.random.default_rng(8)
    A = rng.normal(size=(6, 6))
    A[:, 5] = A[:, 4]
    A = _f32(A)
    b = _f32(np.ones(6))
    x = np.ones(6, np.float32)
    assert oc.lib().oracle_qr_solve(A.ctypes.data, b.ctypes.data, 6, 6, x.ctypes.data) == 0
    assert (x == 0).all()
    # an exactly zero column divides 0 by 0 inside the Householder step: NaN result, which is
    # what the reference's NaN guard (laserOdometry.cpp:799-811) exists for
    Z = _f32(np.zeros((6, 6)))
    assert oc.lib().oracle_qr_solve(Z.ctypes.data, b.ctypes.data, 6, 6, x.ctypes.data) == 1
    assert np.isnan(x).all()


@pytest.mark.parametrize("n", [3, 6])
def test_jacobi_eigen(oc, n):
    rng = np.random.default_rng(4)
    for _ in range(50):
        M = rng.normal(size=(n, n))
        A = _f32(M @ M.T)
        W = np.zeros(n, np.float32)
        V = np.zeros((n, n), np.float32)
        oc.lib().oracle_jacobi(A.ctypes.data, n, W.ctypes.data, V.ctypes.data)
        ev, evec = np.linalg.eigh(A.astype(np.float64))
        ev, evec = ev[::-1], evec[:, ::-1]
        assert np.all(np.diff(W) <= 0)                       # descending (cv::eigen)
        assert np.abs(W - ev).max() <= 1e-4 * max(1.0, ev.max())
        for i in range(n):                                   # rows = eigenvectors, up to sign
            if ev[i] - (ev[i + 1] if i + 1 < n else -1e9) > 1e-2 * ev.max():
                c = abs(float(np.dot(V[i], evec[:, i])))
                assert c > 1 - 1e-3


def _normal_matrices(rng, count):
    """AtA-like 6x6 float matrices (sums of weighted rows with rotation / translation columns of
    different scales), a quarter each: generic, one direction nearly removed, one column shrunk,
    rescaled by 1e-2..1e2"""
    for trial in range(count):
        m = int(rng.integers(20, 3000))
        J = rng.standard_normal((m, 6))
        J[:, :3] *= rng.uniform(0.1, 30)
        w = rng.uniform(0, 1, m)
        kind = trial % 4
        if kind == 1:
            d = rng.standard_normal(6)
            d /= np.linalg.norm(d)
            J -= np.outer(J @ d, d) * rng.uniform(0.9, 1.0)
        elif kind == 2:
            J[:, rng.integers(0, 6)] *= rng.uniform(1e-3, 1e-1)
        elif kind == 3:
            J *= rng.uniform(1e-2, 1e2)
        A = (J * w[:, None]).T @ J
        yield _f32((A + A.T) / 2)


def _certified(A, thr):
    """numpy restatement of loamla::nondegenerate_certified (csrc/dev_common.hpp)"""
    A = A.astype(np.float64)
    nrm = np.abs(A).sum(1).max()
    if not nrm < 1e30:
        return False
    M = A - (thr + nrm * 2.0 ** -14) * np.eye(6)
    L = np.zeros((6, 6))
    d = np.zeros(6)
    for j in range(6):
        dj = M[j, j] - sum(L[j, k] * L[j, k] * d[k] for k in range(j))
        if not dj > 0:
            return False
        d[j] = dj
        for i in range(j + 1, 6):
            L[i, j] = (M[i, j] - sum(L[i, k] * L[j, k] * d[k] for k in range(j))) / dj
    return True


def test_jacobi_eigen_error_bound(oc):
    """the bound behind skipping the iteration-0 eigen-analysis when it cannot change the outcome
    (loamla::nondegenerate_certified): cv::eigen's float Jacobi (the oracle's restatement) returns
    eigenvalues within 2.4 eps_f ||A||_inf of the exact ones on normal-equation-like matrices; the
    certificate's margin, 2^-14 ||A||_inf ~ 512 eps_f, must stay >= 16x the worst error seen"""
    rng = np.random.default_rng(11)
    worst = 0.0
    W = np.zeros(6, np.float32)
    V = np.zeros((6, 6), np.float32)
    for A in _normal_matrices(rng, 4000):
        oc.lib().oracle_jacobi(A.ctypes.data, 6, W.ctypes.data, V.ctypes.data)
        lam = np.linalg.eigvalsh(A.astype(np.float64))
        worst = max(worst, np.abs(np.sort(W.astype(np.float64)) - lam).max() / np.abs(A.astype(np.float64)).sum(1).max())
    assert worst * 16 <= 2.0 ** -14, worst


@pytest.mark.parametrize("thr", [10.0, 100.0])
def test_nondegenerate_certificate_decides_like_jacobi(oc, thr):
    """whenever the certificate holds, the reference's test (smallest cv::eigen eigenvalue >= thr,
    src/laserOdometry.cpp:776-783, src/laserMapping.cpp:933-940) finds no degenerate direction;
    matrices placed just below the threshold are not certified, and those just above only when
    their norm leaves the margin below the gap"""
    rng = np.random.default_rng(12)
    W = np.zeros(6, np.float32)
    V = np.zeros((6, 6), np.float32)
    n_cert = 0
    mats = list(_normal_matrices(rng, 1500))
    below = []
    for i, A in enumerate(mats[:300]):   # the smallest eigenvalue moved to thr * (1 +- 1e-3)
        ev, Q = np.linalg.eigh(A.astype(np.float64))
        ev[0] = thr * (1 + (-1e-3 if i % 2 else 1e-3))
        mats.append(_f32(Q @ np.diag(np.sort(ev)) @ Q.T))
        if i % 2:
            below.append(mats[-1])
    for A in mats:
        oc.lib().oracle_jacobi(A.ctypes.data, 6, W.ctypes.data, V.ctypes.data)
        if _certified(A, thr):
            n_cert += 1
            assert W[5] >= thr, (W, thr)
    for A in below:
        assert not _certified(A, thr)
    assert n_cert > 200
    assert not _certified(np.full((6, 6), np.nan, np.float32), thr)


def test_lu_inverse(oc):
    rng = np.random.default_rng(5)
    for _ in range(50):
        A = _f32(rng.normal(size=(6, 6)) + np.eye(6) * 3)
        inv = np.zeros((6, 6), np.float32)
        assert oc.lib().oracle_lu_inv(A.ctypes.data, 6, inv.ctypes.data) == 1
        assert np.abs(inv @ A - np.eye(6)).max() < 1e-4


def test_pose_message_round_trip(oc):
    rng = np.random.default_rng(6)
    for _ in range(500):
        p = _f32(np.concatenate([rng.uniform(-1.2, 1.2, 3), rng.uniform(-100, 100, 3)]))
        out = np.zeros(6, np.float32)
        oc.lib().oracle_pose_through_msg(p.ctypes.data, out.ctypes.data)
        assert np.abs(out - p).max() <= 4e-7 * max(1.0, np.abs(p[:3]).max())
        np.testing.assert_array_equal(out[3:], p[3:])
