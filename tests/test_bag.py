"""Recorded-sweep ingest (include/loam/loam_bag.h): rosbag v2.0 reading (uncompressed / bz2 / lz4
chunks), sensor_msgs/PointCloud2 (velodyne PointXYZIR zero-copy, other layouts packed by field
name, NaN points passed through) and sensor_msgs/Imu, checked against bags written by
tests/bagwriter.py; host-only (no GPU), except the replay test, which runs the synthetic stream
through the engine from a bag and from arrays and requires identical poses."""
import importlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bagwriter as bw  # noqa: E402


@pytest.fixture(scope="module")
def rb(loam):
    return importlib.import_module("loam_velodyne-1_amd.rosbag")


def _cloud(seed, n=1000, nan=0):
    rng = np.random.default_rng(seed)
    p = rng.uniform(-30, 30, (n, 4)).astype(np.float32)
    p[:, 3] = rng.uniform(0, 100, n)
    if nan:
        p[rng.choice(n, nan, replace=False), :3] = np.nan
    return p


def _messages():
    msgs = []
    for k in range(6):
        t = 100.0 + 0.1 * k
        for j in range(5):
            ti = t + 0.02 * j
            msgs.append(("/imu/data", "sensor_msgs/Imu", ti, bw.imu(ti, [0.0, 0.0, np.sin(ti), np.cos(ti)], [0.1 * j, 9.81, -0.2])))
        msgs.append(("/velodyne_points", "sensor_msgs/PointCloud2", t + 0.05, bw.pointcloud2(_cloud(k), t, seq=k)))
    return msgs


@pytest.mark.parametrize("comp", ["none", "bz2", "lz4", ["none", "bz2", "lz4"]])
def test_bag_round_trip(rb, tmp_path, comp):
    msgs = _messages()
    path = tmp_path / "a.bag"
    bw.write_bag(path, msgs, chunk_messages=7, compression=comp)
    got = list(rb.Bag(path))
    assert len(got) == len(msgs)
    for (t0, ty0, s0, p0), (t1, ty1, s1, p1) in zip(msgs, got):
        assert (t0, ty0) == (t1, ty1)
        assert abs(s0 - s1) < 1e-6
        assert p0 == p1


def test_pointcloud2_velodyne_layout_zero_copy(rb):
    p = _cloud(3, n=2000, nan=17)
    stamp, pts, pc = rb.parse_pc2(bw.pointcloud2(p, 12.25, dense=False))
    assert abs(stamp - 12.25) < 1e-9
    assert (pc.point_step, pc.off_x, pc.off_y, pc.off_z, pc.off_intensity, pc.off_ring) == (32, 0, 4, 8, 16, 20)
    assert pc.is_dense == 0
    np.testing.assert_array_equal(pts, p)  # NaN positions equal too (assert_array_equal treats NaN == NaN)


def test_pointcloud2_other_layout_packed(rb):
    p = _cloud(4, n=777)
    _, pts, pc = rb.parse_pc2(bw.pointcloud2(p, 1.0, layout="shuffled"))
    assert (pc.off_x, pc.off_y, pc.off_z, pc.off_intensity, pc.off_ring) == (4, 8, 12, 0, -1)
    np.testing.assert_array_equal(pts, p)


def _pc2_by_spec(pts, sec, nsec, frame="velodyne"):
    """sensor_msgs/PointCloud2 serialized from the ROS1 message definition itself (not through
    tests/bagwriter.py): Header {uint32 seq, time stamp (uint32 sec, nsec), string frame_id},
    uint32 height, width, PointField[] {string name, uint32 offset, uint8 datatype (7 = FLOAT32,
    4 = UINT16), uint32 count}, bool is_bigendian, uint32 point_step, row_step, uint8[] data,
    bool is_dense; little-endian, strings and arrays length-prefixed with a uint32.  Velodyne layout:
    x, y, z, pad, intensity at 16, ring (uint16) at 20, point_step 32."""
    import struct
    def string(t):
        return struct.pack("<I", len(t)) + t.encode()
    fields = [("x", 0, 7), ("y", 4, 7), ("z", 8, 7), ("intensity", 16, 7), ("ring", 20, 4)]
    n = pts.shape[0]
    rec = np.zeros((n, 32), np.uint8)
    rec[:, 0:12] = np.ascontiguousarray(pts[:, :3], "<f4").view(np.uint8).reshape(n, 12)
    rec[:, 16:20] = np.ascontiguousarray(pts[:, 3], "<f4").view(np.uint8).reshape(n, 4)
    rec[:, 20:22] = (np.arange(n) % 16).astype("<u2").view(np.uint8).reshape(n, 2)
    out = struct.pack("<III", 7, sec, nsec) + string(frame) + struct.pack("<II", 1, n)
    out += struct.pack("<I", len(fields)) + b"".join(string(nm) + struct.pack("<IBI", o, dt, 1) for nm, o, dt in fields)
    out += struct.pack("<BII", 0, 32, 32 * n) + struct.pack("<I", 32 * n) + rec.tobytes() + struct.pack("<B", 0)
    return out


def test_pointcloud2_wire_format_by_spec(rb):
    """the reader against a message packed straight from the ROS1 PointCloud2 definition"""
    p = _cloud(8, n=321, nan=5)
    m = _pc2_by_spec(p, 1234, 500000000)
    stamp, pts, pc = rb.parse_pc2(m)
    assert stamp == 1234.5
    assert (pc.width, pc.height, pc.point_step, pc.row_step) == (321, 1, 32, 32 * 321)
    assert (pc.off_x, pc.off_y, pc.off_z, pc.off_intensity, pc.off_ring) == (0, 4, 8, 16, 20)
    assert (pc.is_bigendian, pc.is_dense) == (0, 0)
    np.testing.assert_array_equal(pts, p)


def test_pc2_cloud_in_reads_message_in_place(rb, tmp_path):
    """rosbag.pc2_cloud_in (the replay path): a velodyne-layout cloud is handed over as a strided
    view of the bag reader's own message buffer (no copy), another layout packed into scratch"""
    import ctypes
    p, q = _cloud(9, n=500, nan=3), _cloud(10, n=200)
    path = tmp_path / "z.bag"
    bw.write_bag(path, [("/velodyne_points", "sensor_msgs/PointCloud2", 1.0, _pc2_by_spec(p, 1, 0)),
                        ("/velodyne_points", "sensor_msgs/PointCloud2", 2.0, bw.pointcloud2(q, 2.0, layout="shuffled"))],
                 chunk_messages=1, compression="lz4")
    seen = 0
    for _topic, _ty, _st, data, size in rb.Bag(path).views():
        stamp, ci, keep = rb.pc2_cloud_in(data, size)
        ref = p if seen == 0 else q
        assert ci.count == ref.shape[0]
        if seen == 0:
            assert keep is None and ci.stride_bytes == 32 and data <= ci.data < data + size
        else:
            assert keep is not None and ci.data == keep.ctypes.data and ci.stride_bytes == 16
        raw = np.frombuffer(ctypes.string_at(ci.data, ci.count * ci.stride_bytes), np.uint8)
        xyz = raw.reshape(ci.count, ci.stride_bytes)[:, :12].copy().view(np.float32)
        np.testing.assert_array_equal(xyz, ref[:, :3])
        seen += 1
    assert seen == 2


def test_pointcloud2_rejects_non_float32_xyz(rb, loam):
    with pytest.raises(loam.LoamError) as e:
        rb.parse_pc2(bw.pointcloud2(_cloud(5, n=10), 1.0, layout="xyz_f64"))
    assert e.value.code == loam.LOAM_E_INVAL


def test_pointcloud2_truncated(rb, loam):
    m = bw.pointcloud2(_cloud(6, n=50), 1.0)
    with pytest.raises(loam.LoamError):
        rb.parse_pc2(m[:-40])


def test_imu_parse(rb):
    t, q, a = rb.parse_imu(bw.imu(3.5, [0.1, -0.2, 0.3, 0.9], [1.0, 9.8, -0.5]))
    assert abs(t - 3.5) < 1e-9
    np.testing.assert_array_equal(q, [0.1, -0.2, 0.3, 0.9])
    np.testing.assert_array_equal(a, [1.0, 9.8, -0.5])


def test_not_a_bag(rb, loam, tmp_path):
    path = tmp_path / "x.bag"
    path.write_bytes(b"#ROSBAG V1.2\n" + b"\0" * 100)
    with pytest.raises(loam.LoamError) as e:
        rb.Bag(path)
    assert e.value.code == loam.LOAM_E_INVAL


def test_truncated_bag(rb, loam, tmp_path):
    path = tmp_path / "t.bag"
    bw.write_bag(path, _messages(), chunk_messages=40)
    data = path.read_bytes()
    path.write_bytes(data[:len(data) // 2])
    with pytest.raises(loam.LoamError):
        list(rb.Bag(path))


@pytest.mark.gpu
def test_chain_sweep_cloud_in_registered(loam, sg):
    """loam_chain_sweep fed a loam_cloud_in view (32-B velodyne records, as rosbag.pc2_cloud_in hands
    them over) with the registered cloud requested: the same poses and registered clouds as the
    array path (the registered cloud is sized from the view's count)"""
    sweeps = sg.stream_sweeps(8, 1)
    cfg = loam.default_config(system_delay=1)
    a, b = loam.Engine(cfg), loam.Engine(cfg)
    mapped = 0
    for k, s in enumerate(sweeps):
        rec = np.zeros((s.shape[0], 8), np.float32)  # x, y, z, pad, intensity, ring, pad, pad
        rec[:, :3] = s[:, :3]
        ci = loam.CloudIn(rec.ctypes.data, rec.shape[0], 32)
        ra = a.chain_sweep(s, stamp=0.1 * k, registered=True)
        rb_ = b.chain_sweep(ci, stamp=0.1 * k, registered=True)
        assert ra[:2] == rb_[:2], k
        for x, y in zip(ra[2:], rb_[2:]):
            assert (x is None) == (y is None), k
            if x is not None:
                np.testing.assert_array_equal(x, y)
        mapped += ra[3] is not None
    assert mapped >= 3


@pytest.mark.gpu
def test_replay_matches_array_path(rb, loam, sg, tmp_path):
    """Config 3 sweeps written to a bag (velodyne layout, bz2 chunks) and replayed: the same poses as
    feeding the arrays to the node path directly (the ingest is lossless)."""
    sweeps = sg.stream_sweeps(14, 1)
    msgs = [("/velodyne_points", "sensor_msgs/PointCloud2", 0.1 * k + 0.05, bw.pointcloud2(s, 0.1 * k, seq=k))
            for k, s in enumerate(sweeps)]
    path = tmp_path / "s.bag"
    bw.write_bag(path, msgs, chunk_messages=4, compression="bz2")
    cfg = loam.default_config(system_delay=2)
    got = rb.replay(path, loam.Engine(cfg))
    eng = loam.Engine(cfg)
    odo, mapped = [], []
    for k, s in enumerate(sweeps):
        rc, f = eng.scan_registration(s, stamp=0.1 * k)
        if rc != 0:
            continue
        pub, pose, cl, sl, full = eng.odometry(f, stamp=0.1 * k)
        if pub & 1:
            odo.append(pose)
        if pub == 7:
            mapped.append(eng.mapping(pose, cl, sl, full, stamp=0.1 * k)[0])
    assert got["sweeps"] == len(sweeps)
    assert len(got["odometry"]) == len(odo) > 5 and len(got["mapping"]) == len(mapped) > 2
    np.testing.assert_array_equal(np.array([p for _, p in got["odometry"]]), np.array(odo))
    np.testing.assert_array_equal(np.array([p for _, p in got["mapping"]]), np.array(mapped))


@pytest.mark.gpu
def test_replay_matches_oracle(rb, loam, oc, sg, tmp_path):
    """A bag as the reference's input (src/scanRegistration.cpp:211-229, :638-660): /velodyne_points
    in the velodyne layout with NaN returns (is_dense = false: pcl::fromROSMsg keeps them,
    removeNaNFromPointCloud drops them) and /imu/data interleaved at 100 Hz, lz4 chunks.  The bag
    replayed through the engine equals the oracle fed the same decoded messages, every
    /laser_odom_to_init and /aft_mapped_to_init pose bit for bit."""
    sweeps = sg.stream_sweeps(16, 1, t0=0.0)
    imus = sg.imu_stream(-0.5, 1.7, seed=1)
    rng = np.random.default_rng(5)
    T0 = 10.0   # ROS stamps are unsigned: the stream's clock starts 10 s into the bag
    msgs, j = [], 0
    for k, s in enumerate(sweeps):
        while j < len(imus) and imus[j][0] <= 0.1 * (k + 1):
            t, q, a = imus[j]
            msgs.append(("/imu/data", "sensor_msgs/Imu", T0 + t, bw.imu(T0 + t, q, a)))
            j += 1
        s = s.copy()
        s[rng.choice(s.shape[0], 300, replace=False), :3] = np.nan
        msgs.append(("/velodyne_points", "sensor_msgs/PointCloud2", T0 + 0.1 * k + 0.1,
                     bw.pointcloud2(s, T0 + 0.1 * k, seq=k, dense=False)))
    path = tmp_path / "imu.bag"
    bw.write_bag(path, msgs, chunk_messages=25, compression="lz4")
    cfg = dict(system_delay=2)
    got = rb.replay(path, loam.Engine(loam.default_config(**cfg)))
    ref = rb.replay(path, oc.Oracle(oc.default_config(**cfg)))
    assert got["sweeps"] == ref["sweeps"] == len(sweeps)
    assert len(got["odometry"]) == len(ref["odometry"]) > 10 and len(got["mapping"]) == len(ref["mapping"]) > 5
    for (tg, pg), (to, po) in zip(got["odometry"] + got["mapping"], ref["odometry"] + ref["mapping"]):
        assert tg == to
        np.testing.assert_array_equal(pg, po)


def _mutations(data, rng, n):
    """n corrupted copies of a byte string: bit flips, overwritten 32-bit length fields, truncations,
    inserted / deleted ranges (the reader parses untrusted bytes: it must fail with an error code,
    never read out of bounds — tools/asan_suite.sh runs this under AddressSanitizer)."""
    out = []
    for _ in range(n):
        b = bytearray(data)
        kind = rng.integers(5)
        if kind == 0:
            for _ in range(rng.integers(1, 8)):
                b[rng.integers(len(b))] ^= 1 << rng.integers(8)
        elif kind == 1:
            at = int(rng.integers(0, len(b) - 4))
            v = int(rng.choice([0, 1, 0x7fffffff, 0xffffffff, len(b), int(rng.integers(0, 1 << 32))]))
            b[at:at + 4] = v.to_bytes(4, "little")
        elif kind == 2:
            b = b[:int(rng.integers(0, len(b)))]
        elif kind == 3:
            at = int(rng.integers(0, len(b)))
            b[at:at] = bytes(rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8))
        else:
            at = int(rng.integers(0, len(b)))
            del b[at:at + int(rng.integers(1, 64))]
        out.append(bytes(b))
    return out


@pytest.mark.parametrize("comp", ["none", "bz2", "lz4"])
def test_bag_fuzz_no_crash(rb, loam, tmp_path, comp):
    path = tmp_path / "f.bag"
    msgs = _messages()[:14]
    bw.write_bag(path, msgs, chunk_messages=5, compression=comp)
    rng = np.random.default_rng({"none": 1, "bz2": 2, "lz4": 3}[comp])
    ok = bad = 0
    for k, b in enumerate(_mutations(path.read_bytes(), rng, 150)):
        q = tmp_path / f"m{k}.bag"
        q.write_bytes(b)
        try:
            for _topic, ty, _s, payload in rb.Bag(q):
                try:
                    if ty == "sensor_msgs/PointCloud2":
                        rb.parse_pc2(payload)
                    elif ty == "sensor_msgs/Imu":
                        rb.parse_imu(payload)
                except loam.LoamError:
                    pass
            ok += 1
        except loam.LoamError:
            bad += 1
    assert ok + bad == 150 and bad > 0


def test_pointcloud2_fuzz_no_crash(rb, loam):
    rng = np.random.default_rng(7)
    base = bw.pointcloud2(_cloud(8, n=64, nan=3), 2.0, seq=3)
    for m in _mutations(base, rng, 400) + _mutations(bw.pointcloud2(_cloud(9, n=40), 1.0, layout="shuffled"), rng, 200):
        try:
            _, pts, pc = rb.parse_pc2(m)
            assert pts.shape[0] == pc.width * pc.height
        except loam.LoamError:
            pass
    for m in _mutations(bw.imu(3.5, [0.1, -0.2, 0.3, 0.9], [1.0, 9.8, -0.5]), rng, 200):
        try:
            rb.parse_imu(m)
        except loam.LoamError:
            pass
