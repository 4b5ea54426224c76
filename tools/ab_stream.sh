#!/bin/bash
# Streaming A/B of experiment builds (configs 2/3 latency legs of bench.py, no batch leg beyond a
# small one): for each library, single_stream (sequential, device chain, pipeline) and latency.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  LOAM_HIP_LIB=$R/$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --latency-runs 30 \
    --batch 8 --global-batch 8 --strong-leg 0 --profile-steps 0 --stream-cpu-sweeps 0 > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));s=d['single_stream'];l=d['latency'];print('$n','seq',round(s['ms_per_sweep'],3),'chain',round(s['device_chain']['ms_per_sweep'],3),'pipe',round(s['pipelined']['ms_per_sweep'],3),'cfg2',round(l['ms_median'],3),'cfg5',round(l['config5']['ms_median'],3))"
done
