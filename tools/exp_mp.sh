#!/bin/bash
# experiment: per-kernel times of diagnostic builds in exp/ (parts of a kernel removed)
for v in base NOSORT NOVGSORT; do
  if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/loam_velodyne-1_amd/exp/libloam_$v.so; fi
  LOAM_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/exp_$v.json 2>&1 || exit 1
done
