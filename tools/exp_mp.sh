#!/bin/bash
# experiment: k_mp_query time with the kNN or the PCA/QR part removed (diagnostic builds in exp/)
for v in base NOGREEDY NOVG NOSORT; do
  if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/loam_velodyne-1_amd/exp/libloam_$v.so; fi
  LOAM_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/exp_$v.json 2>&1 || exit 1
done
