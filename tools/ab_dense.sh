#!/bin/bash
# A/B of launch choices on the config-5 batched leg (bench.py --dense-only); args like tools/ab_share.sh
cd $GRAFT_REPO_ROOT
for C in "$@"; do
  T=()
  if [ "$C" != "default" ]; then IFS=',' read -ra KV <<< "$C"; for kv in "${KV[@]}"; do T+=("--tune=$kv"); done; fi
  n=abd_$(echo "$C" | tr ',=' '_-')
  timeout -k 10 300 python bench.py --dense-only 1 --dense-batch 64 --dense-steps ${STEPS:-5} --cpu-sample 0 "${T[@]}" > gpurun_out/$n.json 2> gpurun_out/$n.err || exit 1
  python - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/{n}.json").read().strip().splitlines()[-1])
k = d["kernel_ms_per_step"]
top = sorted(k.items(), key=lambda kv: -kv[1])[:8]
print(n, round(d["ms_per_step"], 3), round(d["value"]), " ".join(f"{a}={b:.3f}" for a, b in top))
PY
done
