#!/bin/bash
# A/B of the working-tree library against experiment libraries (loam_velodyne-1_amd/exp/NAME.so),
# alternating, at a batch size: BATCH=1024 STEPS=10 N=2 tools/ab_lib.sh head [other ...]
R=$GRAFT_REPO_ROOT; cd $R
B=${BATCH:-1024}
for rep in $(seq ${N:-2}); do
  for L in tree "$@"; do
    if [ $L = tree ]; then unset LOAM_HIP_LIB; else export LOAM_HIP_LIB=$R/loam_velodyne-1_amd/exp/$L.so; fi
    STEPS=${STEPS:-10} BATCH=$B timeout -k 10 300 bash tools/ab_share.sh default | sed "s/^/$L /" || exit 1
  done
done
