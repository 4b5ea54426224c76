#!/bin/bash
# experiment: streaming (configs 3 / 5) timing of the product build and of experiment builds
#   tools/exp_stream.sh NAME...  -> gpurun_out/exps_base.json, gpurun_out/exps_<NAME>.json, exps_base2.json
export STREAM_SWEEPS=${STREAM_SWEEPS:-220} STREAM_CPU_SWEEPS=${STREAM_CPU_SWEEPS:-2}
LOAM_HIP_LIB= timeout -k 10 200 python tools/stream_bench.py > /dev/null 2>&1 || exit 1
for v in base "$@" base2; do
  if [ $v = base ] || [ $v = base2 ]; then L=""; else L=$GRAFT_REPO_ROOT/loam_velodyne-1_amd/exp/libloam_$v.so; fi
  LOAM_HIP_LIB=$L timeout -k 10 200 python tools/stream_bench.py > gpurun_out/exps_$v.json 2>&1 || exit 1
done
