"""Per-frame kernel breakdown of a rocprofv3 kernel trace of the streaming path
(tools/profile_stream.sh): odometry frames (k_od_begin .. k_hash_scatter/k_hash_build of the next
Last clouds) and mapping frames (k_mp_prepare .. k_mp_register).  Diagnostic only.

    python tools/stream_trace.py gpurun_out/prof_stream/st_kernel_trace.csv [first_frame] [frames]
"""
import collections
import csv
import sys


def short(n):
    b = n.replace("(anonymous namespace)", "").split("(")[0].split("::")[-1]
    if "rocprim" in n:
        b = "rocprim"
    return b[:48]


def frames(rows, start_kw, end_kw):
    out, cur = [], None
    for r in rows:
        k = r["Kernel_Name"]
        if start_kw in k:
            cur = [r]
        elif cur is not None:
            cur.append(r)
            if end_kw(k, cur):
                out.append(cur)
                cur = None
    return out


def report(name, fr, first, nf):
    fr = fr[first:first + nf]
    agg, cnt = collections.defaultdict(float), collections.Counter()
    wall = busy = 0.0
    for seg in fr:
        wall += (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            busy += d
            agg[short(r["Kernel_Name"])] += d
            cnt[short(r["Kernel_Name"])] += 1
    n = max(len(fr), 1)
    print(f"{name}: {len(fr)} frames, span {wall / n:.1f} us/frame, kernels busy {busy / n:.1f} us, "
          f"{sum(cnt.values()) / n:.0f} launches")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"  {k:48s} {v / n:8.1f} us  {cnt[k] / n:5.1f} launches")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    report("odometry (k_od_begin .. the next Last index)", frames(
        rows, "k_od_begin", lambda k, c: ("k_hash_scatter" in k or "k_hash_build" in k)
        and sum("k_hash" in x["Kernel_Name"] for x in c) >= (4 if "k_hash_scatter" in k else 2)), first, nf)
    report("mapping", frames(rows, "k_mp_prepare", lambda k, c: "k_mp_register" in k), first, nf)
    report("scan registration", frames(rows, "k_sr_ring_count", lambda k, c: "k_sr_compact" in k), first, nf)


if __name__ == "__main__":
    main()
