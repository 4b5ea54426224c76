"""The mapping's corner fit diagonalises the 5-neighbour covariance with a 3x3 Jacobi
(src/laserMapping.cpp:742, cv::eigen); the device runs it in registers (dev_common.hpp jacobi3_reg),
which must be bit-identical to the generic jacobi<N> the oracle restates (compiled here for the
host)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_jacobi3_reg_is_jacobi3(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "jacobi3_check")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tests", "jacobi3_check.cpp")], check=True, capture_output=True)
    n, bad = map(int, subprocess.run([exe, "1000000"], check=True, capture_output=True, text=True).stdout.split())
    assert n == 1000000 and bad == 0
