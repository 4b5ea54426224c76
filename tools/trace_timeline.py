#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``): per batch step the
wall span, the time some kernel was running (union of dispatch intervals), the idle gaps between
dispatches, and per kernel its dispatches, summed duration and the part of it no other dispatch
overlapped (what shortening that kernel would save at most).

    python tools/trace_timeline.py KERNEL_TRACE.csv [--step-kernel k_sr_ring_count] [--skip N]

Steps are cut at each dispatch of --step-kernel (the first kernel of loam_batch_run); the first
--skip steps (warm-up, profiling pass) are dropped."""
import argparse
import collections
import csv
import json
import re


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)             # drop the argument list
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"^loam::", "", n)
    return n.strip()


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    rows.sort()
    return rows


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def analyse(rows, step_kernel, skip):
    cuts = [i for i, r in enumerate(rows) if r[2].startswith(step_kernel)]
    steps = []
    for a, b in zip(cuts, cuts[1:] + [len(rows)]):
        steps.append(rows[a:b])
    steps = steps[skip:]
    if not steps:
        raise SystemExit("no steps found (step kernel %r)" % step_kernel)
    per = collections.defaultdict(lambda: [0, 0.0, 0.0])  # dispatches, sum us, exclusive us
    walls, busys, queues = [], [], collections.Counter()
    for st in steps:
        t0, t1 = st[0][0], max(r[1] for r in st)
        walls.append((t1 - t0) / 1e3)
        busys.append(union_len([(r[0], r[1]) for r in st]) / 1e3)
        # exclusive time: a 1 us grid over the step is too coarse for 2 us kernels; sweep events
        ev = []
        for i, r in enumerate(st):
            ev.append((r[0], 1, i))
            ev.append((r[1], -1, i))
        ev.sort()
        active = set()
        last = None
        for t, kind, i in ev:
            if last is not None and len(active) == 1:
                (j,) = tuple(active)
                per[st[j][2]][2] += (t - last) / 1e3
            if kind == 1:
                active.add(i)
            else:
                active.discard(i)
            last = t
        for r in st:
            per[r[2]][0] += 1
            per[r[2]][1] += (r[1] - r[0]) / 1e3
            queues[r[3]] += 1
    n = len(steps)
    wall = sum(walls) / n
    busy = sum(busys) / n
    out = {
        "steps": n,
        "wall_us_per_step": round(wall, 1),
        "busy_us_per_step": round(busy, 1),
        "idle_us_per_step": round(wall - busy, 1),
        "dispatches_per_step": round(sum(len(s) for s in steps) / n, 1),
        "queues": dict(queues),
        "kernels": {k: {"dispatches_per_step": round(v[0] / n, 2), "us_per_step": round(v[1] / n, 1),
                        "exclusive_us_per_step": round(v[2] / n, 1), "avg_us": round(v[1] / max(v[0], 1), 2)}
                    for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])},
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step-kernel", default="k_sr_ring_count")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    out = analyse(load(a.trace), a.step_kernel, a.skip)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    print(f"steps {out['steps']}  wall {out['wall_us_per_step']} us  busy {out['busy_us_per_step']} us  "
          f"idle {out['idle_us_per_step']} us  dispatches {out['dispatches_per_step']}")
    print(f"{'kernel':<40} {'n/step':>7} {'us/step':>9} {'excl':>9} {'avg us':>8}")
    for k, v in out["kernels"].items():
        print(f"{k[:40]:<40} {v['dispatches_per_step']:>7} {v['us_per_step']:>9} {v['exclusive_us_per_step']:>9} "
              f"{v['avg_us']:>8}")


if __name__ == "__main__":
    main()
