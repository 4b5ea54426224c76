#!/bin/bash
# Streaming A/B of launch choices (loam_set_tuning) on one library: for each argument
# ("key=value,key=value" or "default") the config-2/3 legs of bench.py (sequential, device chain,
# node pipeline, latency), no CPU legs.  Outputs gpurun_out/abs_<choice>.json.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for C in "$@"; do
  T=()
  if [ "$C" != "default" ]; then IFS=',' read -ra KV <<< "$C"; for kv in "${KV[@]}"; do T+=("--tune=$kv"); done; fi
  n=abs_$(echo "$C" | tr ',=' '_-')
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --latency-runs 30 --batch 8 --global-batch 8 \
    --strong-leg 0 --profile-steps 0 --stream-cpu-sweeps 0 --dense-batch 0 --fed-leg 0 "${T[@]}" \
    > gpurun_out/$n.json 2> gpurun_out/$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/$n.json'));s=d['single_stream'];l=d['latency'];print('$n','seq',round(s['ms_per_sweep'],3),'chain',round(s['device_chain']['ms_per_sweep'],3),'pipe',round(s['pipelined']['ms_per_sweep'],3),'cfg2',round(l['ms_median'],3),'cfg5',round(l['config5']['ms_median'],3))"
done
