"""Input scenarios that drive reference branches the default synthetic streams never reach
(shared by the oracle's CPU tests and the GPU parity tests).

  * pose jumps fed to the mapping node: cube-grid recentring on every axis and in both directions
    (src/laserMapping.cpp:446-614, Q23), including jumps longer than the grid (whole lines cleared)
  * ground-only sweeps (a single plane): the iteration-0 degeneracy projection fires in odometry
    (eigenvalue < 10, src/laserOdometry.cpp:770-797) and in mapping (< 100,
    src/laserMapping.cpp:927-954)
  * Last clouds smaller than the next sweep's sharp / flat counts: the Q11 forward window
    (src/laserOdometry.cpp:486, :598) runs to the end of CornerLast / SurfLast
  * a corner pair at one position on two rings in the Last cloud: point-to-line with l12 = 0 gives
    NaN coefficients that pass `s > 0.1 && ld2 != 0` at iterations < 5, so the NaN guard
    (src/laserOdometry.cpp:799-811, Q16) skips every update of that frame
"""
import numpy as np

# mapping-frame pose offsets (metres, added to the odometry translation) for the recentring
# stream: +x (1 shift down), back, +y, back, -z (up), back, -y, back, -x beyond the grid (16
# shifts up: the origin's content is cleared), then the way back (8 down), +z (12), back
GRID_JUMPS = [(0, 0, 0)] * 4 + [(400, 0, 0), (0, 0, 0), (0, 140, 0), (0, 0, 0), (0, 0, -420), (0, 0, 0),
                                (0, -150, 0), (0, 0, 0), (-1100, 0, 0), (0, 0, 0), (0, 0, 900), (0, 0, 0)]


def ground_only(raw, z_max=-1.0):
    """the returns of a sweep below z_max in the sensor frame (the floor at -1.5 m): one plane"""
    return raw[raw[:, 2] < z_max]


def duplicate_corners(less_sharp, n_sharp, every=4, count=10):
    """insert before some lessSharp points (index < the sweep's sharp count, so both the forward
    window, bounded by cornerPointsSharpNum (Q11), and the backward one reach the pair) a copy one
    ring lower (same relTime): after TransformToEnd the two Last points coincide on rings r-1, r"""
    sel = [i for i in range(1, min(n_sharp, less_sharp.shape[0])) if less_sharp[i, 3] >= 1.0]
    sel = set(sel[:every * count:every])
    rows = []
    for i in range(less_sharp.shape[0]):
        if i in sel:
            d = less_sharp[i].copy()
            d[3] -= 1.0
            rows.append(d)
        rows.append(less_sharp[i])
    return np.array(rows, np.float32).reshape(-1, 4), len(sel)


def truncate_last(f, n_corner=14, n_surf=120):
    """keep only the last n_corner lessSharp / n_surf lessFlat points (the highest rings): the next
    sweep's CornerLast / SurfLast are then smaller than its sharp / flat counts (still above the
    L-M gate 10 / 100, src/laserOdometry.cpp:465), so the forward ring windows of Q11, bounded by
    cornerPointsSharpNum / surfPointsFlatNum (:486, :598), run past the Last clouds' ends — the
    reference reads beyond the vector there; engine and oracle both clamp at |Last|"""
    f = dict(f)
    f["less_sharp"] = np.ascontiguousarray(f["less_sharp"][-n_corner:])
    f["less_flat"] = np.ascontiguousarray(f["less_flat"][-n_surf:])
    return f


def run_stream(impl, sweeps, *, mapping=True, jumps=None, inject_nan_at=None, truncate_last_at=(),
               stats=True):
    """scan registration -> odometry -> mapping over `sweeps` with the scenario hooks; returns one
    record per odometry call: published flags, pose, the three odometry clouds, and on mapping
    frames aft / bef / registered / surround plus the branch counters"""
    out = []
    m = 0
    for k, sw in enumerate(sweeps):
        rc, f = impl.scan_registration(sw, stamp=0.1 * k)
        if rc != 0:
            continue
        if inject_nan_at is not None and k == inject_nan_at:
            f = dict(f)
            f["less_sharp"], _ = duplicate_corners(f["less_sharp"], f["sharp"].shape[0])
        if k in truncate_last_at:
            f = truncate_last(f)
        pub, pose, cl, sl, full = impl.odometry(f, stamp=0.1 * k)
        rec = {"k": k, "pub": pub, "pose": pose, "corner_last": cl, "surf_last": sl, "full_end": full,
               "n_sharp": int(f["sharp"].shape[0]), "n_flat": int(f["flat"].shape[0]),
               "n_less_sharp": int(f["less_sharp"].shape[0]), "n_less_flat": int(f["less_flat"].shape[0])}
        if stats:
            s = impl.stats()
            rec["od_deg"], rec["od_nan"] = s["od_degenerate_steps"], s["od_nan_skips"]
            rec["od_iters"] = s["od_iters"]
        if mapping and pub == 7:
            p = pose.copy()
            if jumps is not None:
                p[3:] += np.float32(jumps[m] if m < len(jumps) else (0, 0, 0))
            aft, bef, reg = impl.mapping(p, cl, sl, full, stamp=0.1 * k)
            rec.update(aft=aft, bef=bef, registered=reg, surround=impl.mapping_surround())
            if stats:
                s = impl.stats()
                rec["mp_deg"], rec["mp_shifts"], rec["mp_iters"] = (s["mp_degenerate_steps"], s["mp_grid_shifts"],
                                                                   s["mp_iters"])
            m += 1
        out.append(rec)
    return out
