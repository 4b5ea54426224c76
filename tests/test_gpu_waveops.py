"""The DPP / permlane cross-lane primitives (dev_common.hpp wave_*_x) equal the __shfl forms on
random keys, floats and integers over whole waves and 32-lane halves (tools/mb/waveops_check.hip,
built by loam_velodyne-1_amd/Makefile)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cross_lane_primitives():
    exe = os.path.join(ROOT, "tools", "mb", "waveops_check")
    assert os.path.exists(exe), "build first (make -C loam_velodyne-1_amd)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_wave_qr_solve_bitexact():
    """loamla::qr_solve6_wave (the L-M step's 6x6 QR solve by a whole wave) equals the one-lane
    qr_solve bit for bit on 32768 systems (normal equations at several scales, rank-deficient,
    general, NaN / inf entries; a NaN matches a NaN)."""
    exe = os.path.join(ROOT, "tools", "mb", "qr_wave_check")
    assert os.path.exists(exe), "build first (make -C loam_velodyne-1_amd)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
