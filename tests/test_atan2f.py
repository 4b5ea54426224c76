"""The engine's device atan2f (dev_common.hpp atan2f_fdlibm, compiled here for the host) must be
bit-identical to glibc's atan2f, which the reference's `using std::atan2` binds to
(src/scanRegistration.cpp:53): scan-registration orientation / relTime / intensity depend on it."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_device_atan2f_is_glibc(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "atan2f_check")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(ROOT, "tests", "atan2f_check.cpp")],
                   check=True, capture_output=True)
    n, bad = map(int, subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split())
    assert n == 4000000 and bad == 0
