"""Per-dispatch averages of the PMC counters rocprofv3 collected for one kernel family
(tools/pmc_kernel.sh / tools/pmc_ta.sh outputs), plus the derived shares the DESIGN notes cite.

    python tools/pmc_summary.py NAME CSV [CSV ...] >> OUT.csv
"""
import collections
import csv
import sys


def main():
    name, paths = sys.argv[1], sys.argv[2:]
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            c = r["Counter_Name"]
            tot[c] += float(r["Counter_Value"])
            disp[c].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    avg = {c: tot[c] / max(1, len(disp[c])) for c in tot}
    print(f"# {name}: rocprofv3 --pmc, batch 1024, per dispatch (averaged over {max(len(v) for v in disp.values())} dispatches)")
    for c in sorted(avg):
        print(f"{name},{c},{avg[c]:.1f}")
    if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
        print(f"{name},derived_wait_share,{avg['SQ_WAIT_ANY'] / avg['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        print(f"{name},derived_valu_per_wave,{avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.1f}")
    if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        # a wave64 VALU instruction issues over 2 cycles (MI355X_MICROARCH.md), over 1024 SIMDs x the
        # kernel's cycles (GRBM_GUI_ACTIVE sums the 8 XCDs)
        kc = avg["GRBM_GUI_ACTIVE"] / 8
        print(f"{name},derived_valu_issue_share,{2 * avg['SQ_INSTS_VALU'] / (1024 * kc):.3f}")
        print(f"{name},derived_waves_per_simd,{4 * avg['SQ_WAVE_CYCLES'] / (1024 * kc):.2f}")


if __name__ == "__main__":
    main()
