"""Phase times of k_sr_ringvg's ring VoxelGrid (diagnostic build: tools/build_variant.sh NAME
-DLOAM_VG_PH, then LOAM_HIP_LIB=.../exp/NAME.so python tools/vg_phases.py [P] [steps]).  Prints the
mean shader cycles per ring of: prologue..bbox, runs, nxt, sort, voxel means."""
import ctypes
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
loam = importlib.import_module("loam_velodyne-1_amd")
sg = importlib.import_module("loam_velodyne-1_amd.synthgen")


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    prevs, curs = sg.batch_problems(P, base_seed=1000)
    e = loam.Engine()
    e.batch_upload(prevs, curs)
    e.batch_run()
    e.sync()
    f = loam.lib().loam_diag_vg_phases
    buf = (ctypes.c_ulonglong * 8)()
    f(buf, 1)
    for _ in range(K):
        e.batch_run()
    e.sync()
    f(buf, 0)
    n = max(1, buf[5])
    names = ["bbox", "runs", "nxt", "sort", "means"]
    print(f"rings {n}: " + ", ".join(f"{nm} {buf[i] / n:.0f}" for i, nm in enumerate(names)) + " cycles/ring")
    e.close()


if __name__ == "__main__":
    main()
