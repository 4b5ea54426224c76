#!/bin/bash
# experiment: bench lines of the product build and of experiment builds exp/libloam_<NAME>.so
#   tools/exp_mp.sh NAME...      -> gpurun_out/exp_base.json, gpurun_out/exp_<NAME>.json
# A discarded warm-up run goes first (the first bench on a fresh box runs slower), and the
# product build runs again last (exp_base2.json) to bracket drift.
LOAM_HIP_LIB= timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --profile-steps 1 --stream-sweeps 0 > /dev/null 2>&1 || exit 1
for v in base "$@" base2; do
  if [ $v = base ] || [ $v = base2 ]; then L=""; else L=$GRAFT_REPO_ROOT/loam_velodyne-1_amd/exp/libloam_$v.so; fi
  LOAM_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --stream-sweeps 0 > gpurun_out/exp_$v.json 2>&1 || exit 1
done
