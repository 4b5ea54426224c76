"""Stand-in engine for the bench harness tests on CPU-only machines (bench.py LOAM_BENCH_ENGINE).

Test infrastructure: it exercises bench.py's rank spawning, sharding, timing and pose gathering
without a GPU.  Its "poses" are a cheap deterministic function of each problem's two sweeps
(centroids), so a gathered result can be checked against a single-process run.  It is never used
for a measurement."""
import numpy as np

STAT_KEYS = ("n_raw", "n_ring", "n_sharp", "n_less_sharp", "n_flat", "n_less_flat", "od_iters",
             "od_assoc_rounds", "od_rows_sum", "od_corner_last", "od_surf_last", "od_queries",
             "od_assoc_points", "mp_iters", "mp_rows_sum", "mp_stack", "mp_map_points",
             "mp_map_valid_points", "mp_stack_iters", "mp_fits", "od_query_iters", "od_row_evals",
             "bytes_sr", "bytes_od", "bytes_mp", "od_degenerate_steps", "od_nan_skips",
             "mp_degenerate_steps", "mp_grid_shifts", "mp_nn_candidates", "mp_nn_cells",
             "od_assoc_gathered", "od_assoc_boxes")


def poses_of(prev, cur):
    a = np.asarray(prev, np.float32)[:, :3].mean(axis=0)
    b = np.asarray(cur, np.float32)[:, :3].mean(axis=0)
    return np.concatenate([a, b]).astype(np.float32), np.concatenate([b, a]).astype(np.float32)


class Engine:
    def __init__(self, device=0):
        self.n = 0

    def batch_upload(self, prevs, curs):
        self.n = len(prevs)
        self.res = [poses_of(p, c) for p, c in zip(prevs, curs)]

    def batch_run(self):
        pass

    def sync(self):
        pass

    def batch_download(self):
        od = np.stack([r[0] for r in self.res])
        aft = np.stack([r[1] for r in self.res])
        st = {k: self.n for k in STAT_KEYS}
        return od, aft, st

    def set_profiling(self, on):
        pass

    def kernel_times(self):
        return {"k_mp_nnfit": (1.0, 10), "k_od_assoc": (0.5, 5)}

    def close(self):
        pass
