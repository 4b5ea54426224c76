"""Test infrastructure: a minimal rosbag v2.0 writer (chunks stored uncompressed, bz2 or lz4) and the
ROS1 serialisation of sensor_msgs/PointCloud2 and sensor_msgs/Imu, to build fixture bags for the
reader in libloam_hip.so (include/loam/loam_bag.h).  Written from the published rosbag v2.0 format
(records = u32 header length, "name=value" fields, u32 data length, data; op codes 0x02 message,
0x03 bag header, 0x04 index, 0x05 chunk, 0x06 chunk info, 0x07 connection)."""
import bz2
import ctypes
import struct

import numpy as np

FLOAT32, FLOAT64, UINT16 = 7, 8, 4  # sensor_msgs/PointField datatypes


def _field(name, value):
    b = name.encode() + b"=" + value
    return struct.pack("<I", len(b)) + b


def _record(fields, data):
    hdr = b"".join(_field(k, v) for k, v in fields)
    return struct.pack("<I", len(hdr)) + hdr + struct.pack("<I", len(data)) + data


def _string(s):
    b = s.encode()
    return struct.pack("<I", len(b)) + b


def _header(seq, stamp, frame):
    sec = int(np.floor(stamp))
    nsec = int(round((stamp - sec) * 1e9))
    if nsec >= 1000000000:
        sec, nsec = sec + 1, nsec - 1000000000
    return struct.pack("<III", seq, sec, nsec) + _string(frame)


def pointcloud2(points, stamp, layout="velodyne", seq=0, dense=True):
    """points: (n, 4) float32 x, y, z, intensity.  layout "velodyne" = PointXYZIR (x, y, z at 0/4/8,
    intensity at 16, uint16 ring at 20, point_step 32); "shuffled" = intensity, x, y, z at 0/4/8/12
    (point_step 16); "xyz_f64" = x, y, z as FLOAT64 (not accepted by the reader)."""
    p = np.asarray(points, np.float32)
    n = p.shape[0]
    if layout == "velodyne":
        fields = [("x", 0, FLOAT32), ("y", 4, FLOAT32), ("z", 8, FLOAT32), ("intensity", 16, FLOAT32),
                  ("ring", 20, UINT16)]
        step = 32
        rec = np.zeros((n, 32), np.uint8)
        rec[:, 0:12] = p[:, :3].view(np.uint8).reshape(n, 12)
        rec[:, 16:20] = p[:, 3:4].copy().view(np.uint8).reshape(n, 4)
    elif layout == "shuffled":
        fields = [("intensity", 0, FLOAT32), ("x", 4, FLOAT32), ("y", 8, FLOAT32), ("z", 12, FLOAT32)]
        step = 16
        rec = np.ascontiguousarray(p[:, [3, 0, 1, 2]]).view(np.uint8).reshape(n, 16)
    elif layout == "xyz_f64":
        fields = [("x", 0, FLOAT64), ("y", 8, FLOAT64), ("z", 16, FLOAT64)]
        step = 24
        rec = p[:, :3].astype(np.float64).view(np.uint8).reshape(n, 24)
    else:
        raise ValueError(layout)
    out = _header(seq, stamp, "velodyne") + struct.pack("<II", 1, n)
    out += struct.pack("<I", len(fields))
    for name, off, dt in fields:
        out += _string(name) + struct.pack("<IBI", off, dt, 1)
    data = rec.tobytes()
    out += struct.pack("<BII", 0, step, step * n) + struct.pack("<I", len(data)) + data
    out += struct.pack("<B", 1 if dense else 0)
    return out


def imu(stamp, quat_xyzw, lin_acc, seq=0):
    z9 = [0.0] * 9
    return (_header(seq, stamp, "imu") + struct.pack("<4d", *quat_xyzw) + struct.pack("<9d", *z9) +
            struct.pack("<3d", 0.0, 0.0, 0.0) + struct.pack("<9d", *z9) + struct.pack("<3d", *lin_acc) +
            struct.pack("<9d", *z9))


TYPES = {"sensor_msgs/PointCloud2": "1158d486dd51d683ce2f1be655c3c181", "sensor_msgs/Imu": "6a62c6daae103f4ff57a132d6f95cec2"}


def _lz4_frame(raw):
    L = ctypes.CDLL("liblz4.so.1")
    L.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    L.LZ4F_compressFrameBound.argtypes = [ctypes.c_size_t, ctypes.c_void_p]
    L.LZ4F_compressFrame.restype = ctypes.c_size_t
    L.LZ4F_compressFrame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    cap = L.LZ4F_compressFrameBound(len(raw), None)
    dst = ctypes.create_string_buffer(cap)
    src = ctypes.create_string_buffer(raw, len(raw))
    n = L.LZ4F_compressFrame(dst, cap, src, len(raw), None)
    return dst.raw[:n]


def write_bag(path, messages, chunk_messages=8, compression="none"):
    """messages: list of (topic, type, stamp, payload bytes) in file order; chunks of
    chunk_messages messages, each compressed with `compression` (a str, or a list cycled per chunk)."""
    comps = [compression] if isinstance(compression, str) else list(compression)
    conns = {}
    chunks = []
    for c0 in range(0, len(messages), chunk_messages):
        inner = b""
        for topic, mtype, stamp, payload in messages[c0:c0 + chunk_messages]:
            if topic not in conns:
                cid = len(conns)
                conns[topic] = (cid, mtype)
                chdr = b"".join(_field(k, v.encode()) for k, v in
                                [("topic", topic), ("type", mtype), ("md5sum", TYPES.get(mtype, "*")),
                                 ("message_definition", "")])
                inner += _record([("op", b"\x07"), ("conn", struct.pack("<I", cid)), ("topic", topic.encode())], chdr)
            sec = int(np.floor(stamp))
            nsec = int(round((stamp - sec) * 1e9)) % 1000000000
            inner += _record([("op", b"\x02"), ("conn", struct.pack("<I", conns[topic][0])),
                              ("time", struct.pack("<II", sec, nsec))], payload)
        comp = comps[len(chunks) % len(comps)]
        data = {"none": lambda b: b, "bz2": bz2.compress, "lz4": _lz4_frame}[comp](inner)
        chunks.append(_record([("op", b"\x05"), ("compression", comp.encode()), ("size", struct.pack("<I", len(inner)))], data))
    head = _record([("op", b"\x03"), ("index_pos", struct.pack("<Q", 0)), ("conn_count", struct.pack("<I", len(conns))),
                    ("chunk_count", struct.pack("<I", len(chunks)))], b" " * 4096)
    tail = b""  # connection records again after the chunks, as rosbag writes them (with its index)
    for topic, (cid, mtype) in conns.items():
        chdr = b"".join(_field(k, v.encode()) for k, v in [("topic", topic), ("type", mtype)])
        tail += _record([("op", b"\x07"), ("conn", struct.pack("<I", cid)), ("topic", topic.encode())], chdr)
    with open(path, "wb") as f:
        f.write(b"#ROSBAG V2.0\n" + head + b"".join(chunks) + tail)
