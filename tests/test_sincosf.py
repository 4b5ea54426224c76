"""The engine's device sinf / cosf (dev_common.hpp sinf_glibc / cosf_glibc, compiled here for the
host) must be bit-identical to glibc's, which scanRegistration's IMU de-skew binds to through
`using std::sin/cos` on floats (src/scanRegistration.cpp:51-53, :111-179)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_device_sincosf_is_glibc(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "sincosf_check")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-fno-builtin", "-o", exe,
                    os.path.join(ROOT, "tests", "sincosf_check.cpp")], check=True, capture_output=True)
    # every 61st float of |x| < 120, both signs (the full sweep, step 3, is 0 mismatches too)
    n, bs, bc = map(int, subprocess.run([exe, "61"], check=True, capture_output=True, text=True).stdout.split())
    assert n > 30000000 and bs == 0 and bc == 0
