#!/bin/bash
# A/B of the config-5 batched leg across libraries (loam_velodyne-1_amd/exp/NAME.so) against the
# working tree, alternating N times:  N=2 tools/ab_dense_lib.sh other [other ...]
R=$GRAFT_REPO_ROOT; cd $R
for rep in $(seq ${N:-2}); do
  for L in tree "$@"; do
    if [ $L = tree ]; then unset LOAM_HIP_LIB; else export LOAM_HIP_LIB=$R/loam_velodyne-1_amd/exp/$L.so; fi
    timeout -k 10 300 bash tools/ab_dense.sh default | sed "s/^/$L /" || exit 1
  done
done
