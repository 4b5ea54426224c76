#!/bin/bash
# A/B of launch choices (loam_set_tuning) at a batch size, one library: for each argument
# ("key=value,key=value" or "default") a short bench line with the per-kernel ms/step.
#   BATCH=128 tools/ab_share.sh default od_fused_max=0 mp_fused_max=0
# Outputs gpurun_out/ab_<BATCH>_<choice>.json; prints one summary line per choice.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B=${BATCH:-128}
for C in "$@"; do
  T=()
  if [ "$C" != "default" ]; then
    IFS=',' read -ra KV <<< "$C"
    for kv in "${KV[@]}"; do T+=("--tune=$kv"); done
  fi
  n=ab_${B}_$(echo "$C" | tr ',=' '_-')
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --cpu-sample 0 --latency-runs 0 \
    --batch $B --global-batch $B --strong-leg 0 --stream-sweeps 0 --dense-batch 0 "${T[@]}" \
    > gpurun_out/$n.json 2> gpurun_out/$n.err || exit 1
  python - "$n" <<'EOF'
import json, sys
n = sys.argv[1]
d = json.load(open(f"gpurun_out/{n}.json"))
k = d["kernel_ms_per_step"]
top = sorted(k.items(), key=lambda kv: -kv[1])[:10]
print(n, round(d["ms_per_step"], 3), round(d["value"]), " ".join(f"{a}={b:.3f}" for a, b in top))
EOF
done
