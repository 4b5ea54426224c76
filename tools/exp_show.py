"""Summarise tools/exp_mp.sh results: ms/step and chosen kernels per variant."""
import json
import sys

names = sys.argv[1].split(",")
kern = sys.argv[2].split(",") if len(sys.argv) > 2 else []
for n in ["base"] + names + ["base2"]:
    try:
        d = json.loads(open(f"gpurun_out/exp_{n}.json").read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(n, "missing", e)
        continue
    k = d["kernel_ms_per_step"]
    print(f"{n:12s} {d['ms_per_step']:7.2f}", " ".join(f"{x}={k.get(x, 0):.3f}" for x in kern))
