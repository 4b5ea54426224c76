"""The 5-NN search lists the buckets of the 27 cells around a query point and offers every point
of them once, without a duplicate test (loam_velodyne-1_amd/csrc/mp.hip knn5_flat): that needs
cell_hash to put the 27 cells in 27 different buckets for every table size the map hash uses
(>= 64 buckets).  tests/cellhash_check.cpp compiles the device function for the host and checks
random cells (signs included) against every table size 2^6 .. 2^20."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_cell_hash_separates_neighbourhoods(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "cellhash_check")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O2", "-o", exe, os.path.join(ROOT, "tests", "cellhash_check.cpp")], check=True,
                   capture_output=True)
    checked, collisions = map(int, subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split())
    assert checked == 3000000 and collisions == 0
