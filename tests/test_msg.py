"""The reference's pose message conventions (include/loam/loam_msg.h), host functions, no GPU:
orientation = (-q.y, -q.z, q.x, q.w) of createQuaternionMsgFromRollPitchYaw(rz, -rx, -ry)
(src/laserOdometry.cpp:858-866, src/laserMapping.cpp:1071-1080, src/transformMaintenance.cpp:163-171),
transformBefMapped in the twist fields (src/laserMapping.cpp:1082-1087), and the handlers' read-back
(src/laserMapping.cpp:304-321, src/transformMaintenance.cpp:147-160,182-203).  Checked bit for bit
against the oracle's restatement of the same tf algebra.  (Thousands of poses: a quaternion
built from separate sin / cos instead of the sincos pair GCC emits differs in ~0.4 % of them.)"""
import ctypes

import numpy as np
import pytest


def _poses(n, seed=3):
    rng = np.random.default_rng(seed)
    p = np.zeros((n, 6), np.float32)
    p[:, :3] = rng.uniform(-3.0, 3.0, (n, 3))
    p[:, 0] = rng.uniform(-1.4, 1.4, n)            # |rx| < pi/2: getRPY's regular branch
    p[:, 3:] = rng.uniform(-500, 500, (n, 3))
    return p


def _oracle_orientation(oc, p):
    q = np.zeros(4, np.float64)
    oc.lib().oracle_msg_orientation(np.ascontiguousarray(p, np.float32).ctypes.data, q.ctypes.data)
    return q


def _oracle_round_trip(oc, p):
    out = np.zeros(6, np.float32)
    pin = np.ascontiguousarray(p, np.float32)
    oc.lib().oracle_pose_through_msg(pin.ctypes.data, out.ctypes.data)
    return out


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_msg_from_pose_matches_oracle(loam, oc, kind):
    frames = {0: b"/laser_odom", 1: b"/aft_mapped", 2: b"/camera"}
    for p in _poses(4000):
        bef = p[::-1].copy()
        m, t = loam.msg_from_pose(kind, p, bef if kind == 1 else None, stamp=12.5)
        np.testing.assert_array_equal(np.array(m.orientation[:]), _oracle_orientation(oc, p))
        np.testing.assert_array_equal(np.array(m.position[:]), p[3:].astype(np.float64))
        assert m.stamp == 12.5 and m.frame_id == b"/camera_init" and m.child_frame_id == frames[kind]
        np.testing.assert_array_equal(np.array(t.rotation[:]), np.array(m.orientation[:]))
        np.testing.assert_array_equal(np.array(t.origin[:]), np.array(m.position[:]))
        if kind == 1:
            np.testing.assert_array_equal(np.array(m.twist_angular[:] + m.twist_linear[:]), bef.astype(np.float64))
        else:
            assert not any(m.twist_angular[:]) and not any(m.twist_linear[:])


def test_round_trip_matches_oracle(loam, oc):
    """publish -> receive = the oracle's pose_through_msg bit for bit; Bef passes through exactly"""
    for p in _poses(8000, seed=11):
        m, _ = loam.msg_from_pose(loam.MSG_AFT_MAPPED, p, p * 0.5)
        back, bef = loam.pose_from_msg(m)
        np.testing.assert_array_equal(back, _oracle_round_trip(oc, p))
        np.testing.assert_array_equal(bef, (p * 0.5).astype(np.float32))
        assert np.abs(back - p).max() < 1e-5          # identity up to rounding away from |rx| = 90 deg


def test_gimbal_branch(loam, oc):
    """|rx| = pi/2 takes getRPY's |m20| >= 1 branch (yaw = 0)"""
    for rx in (np.float32(np.pi / 2), np.float32(-np.pi / 2)):
        p = np.array([rx, 0.3, -0.2, 1, 2, 3], np.float32)
        m, _ = loam.msg_from_pose(loam.MSG_LASER_ODOM, p)
        back, _ = loam.pose_from_msg(m)
        np.testing.assert_array_equal(back, _oracle_round_trip(oc, p))


def test_msg_errors(loam):
    p = loam.Pose6.of(np.zeros(6))
    m, t = loam.OdometryMsg(), loam.TfMsg()
    lib = loam.lib()
    assert lib.loam_msg_from_pose(7, 0.0, ctypes.byref(p), None, ctypes.byref(m), None) == loam.LOAM_E_INVAL
    assert lib.loam_msg_from_pose(1, 0.0, ctypes.byref(p), None, ctypes.byref(m), None) == loam.LOAM_E_INVAL
    assert lib.loam_msg_from_pose(0, 0.0, ctypes.byref(p), None, ctypes.byref(m), None) == loam.LOAM_OK
    assert lib.loam_pose_from_msg(None, ctypes.byref(p), None) == loam.LOAM_E_INVAL
