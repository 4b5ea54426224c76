"""Per-round durations of k_od_assoc from a rocprofv3 kernel trace (diagnostic): the association
runs every 5th odometry iteration (Q10), so within a step its launches are rounds 0..4; round 0 is
the unseeded one.   python tools/assoc_rounds.py KERNEL_TRACE.csv [launches_per_step=5]"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_od_assoc" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 5
acc = collections.defaultdict(list)
for i, r in enumerate(rows):
    acc[i % per].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in sorted(acc):
    v = acc[k][1:] if len(acc[k]) > 2 else acc[k]  # (the first step warms up)
    print(f"round {k}: {sum(v) / len(v):8.1f} us  ({len(v)} launches)")
