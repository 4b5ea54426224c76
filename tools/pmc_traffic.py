"""Per-kernel HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of the
same bench command, corrected as /opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes:
counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled; WRITE_SIZE is taken as is.  Writes profiles/traffic.json (bytes per launch per kernel,
read by bench.py for roofline.traffic) and a per-kernel summary CSV.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT_JSON OUT_CSV
"""
import collections
import csv
import json
import sys


# the VoxelGrid cascade's kernels carry their job as the last template argument (mp.hip vg_run's
# TAG): they are reported per job, under bench.py's names for the two jobs of a step
VG_JOBS = {"0": "vg_stack", "1": "vg_cubes", "2": "vg_surround"}


def short(name):
    base = name.replace("(anonymous namespace)", "").split("(")[0]
    if "rocprim" in base:
        return "rocprim_segmented_radix_sort" if "segmented_radix_sort" in name else "rocprim_other"
    base = base.split("::")[-1]
    if base.startswith(("k_vg_radix<", "k_vg_idx<", "k_vg_big<")):
        # vg_stack<k_vg_idx>: one instantiation of the job's cascade (summed per launch below)
        tag = base.rstrip(">").split(",")[-1].strip()
        return VG_JOBS.get(tag, "vg_other") + "<" + base.split("<")[0] + ">"
    if base.startswith("k_vg_merge<"):
        return "vg_cubes<k_vg_merge>"
    if base.startswith(("k_vg_split<", "k_vg_join<")):  # (the stack job's big-segment split)
        return "vg_stack<" + base.split("<")[0] + ">"
    return base


def load(path):
    """{kernel: [total KiB, launches]}; template instantiations of one kernel (launched together,
    timed as one by bench.py) are summed per launch"""
    inst = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        inst[k][0] += float(r["Counter_Value"])
        inst[k][1] += 1
    # kernels with a profiling (COUNT) variant (k_mp_nnfit<., true>, k_od_assoc<true, ...>): the variant
    # launches in place of the plain one in the bench's profiling pass, so both are dispatches of
    # the same launch: every dispatch of either counts, averaged together
    counted = {k.split("<")[0] for k in inst if "<true" in k}
    counted |= {k.split("<")[0] for k in inst if k.startswith("k_mp_nnfit<")}  # (COUNT last)
    merged = collections.defaultdict(lambda: [0.0, 0])
    for k, (v, n) in inst.items():
        if k.split("<")[0] in counted:
            merged[k.split("<")[0] + "<any>"][0] += v
            merged[k.split("<")[0] + "<any>"][1] += n
    inst = {k: v for k, v in inst.items() if k.split("<")[0] not in counted}
    inst.update(merged)
    agg = collections.defaultdict(lambda: [0.0, 0])
    for k, (v, n) in inst.items():
        base = k.split("<")[0]
        agg[base][0] += v / max(n, 1)   # per launch of this instantiation
        agg[base][1] = 1
    for k in agg:                       # report launches of the first instantiation seen
        agg[k][1] = max(n for kk, (v, n) in inst.items() if kk.split("<")[0] == k)
        agg[k][0] *= agg[k][1]
    return agg


def main():
    fetch, write, out_json, out_csv = sys.argv[1:5]
    f, w = load(fetch), load(write)
    res = {}
    rows = []
    for k in sorted(set(f) | set(w)):
        fk, fn = f.get(k, [0.0, 0])
        wk, wn = w.get(k, [0.0, 0])
        fb = 2.0 * fk * 1024 / max(fn, 1)
        wb = wk * 1024 / max(wn, 1)
        res[k] = fb + wb
        rows.append((k, fn, fk * 1024 / max(fn, 1), fb, wb, fb + wb))
    # bench.py's stage names over several kernels, each launched once per launch of the stage: the
    # ring sort (fused, or count + scatter), the selection (picks, ring VoxelGrid, the fallbacks) and the
    # odometry rows (the moments form in batches)
    groups = {"k_sr_ring_sort": ["k_sr_ring_fused", "k_sr_ring_count", "k_sr_ring_scatter"],
              "k_sr_select": ["k_sr_pick", "k_sr_ringvg", "k_sr_select"]}
    for g, ks in groups.items():
        if any(k in res for k in ks):
            res[g] = sum(res.get(k, 0.0) for k in ks)
    if "k_od_rows_mom" in res and "k_od_rows" not in res:
        res["k_od_rows"] = res["k_od_rows_mom"]
    res["_note"] = ("HBM-side bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B), averaged over "
                    "the dispatches of two separate --pmc passes of bench.py --steps 2 --warmup 1")
    json.dump(res, open(out_json, "w"), indent=1, sort_keys=True)
    with open(out_csv, "w") as o:
        o.write("kernel,launches,fetch_size_bytes_raw,fetch_bytes_x2,write_bytes,traffic_bytes_per_launch\n")
        for r in sorted(rows, key=lambda r: -r[5] * r[1]):
            o.write("%s,%d,%.0f,%.0f,%.0f,%.0f\n" % r)


if __name__ == "__main__":
    main()
