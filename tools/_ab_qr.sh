#!/bin/bash
# A/B: wave QR (default lib) vs one-lane QR (exp/qr1.so): chain and share, alternating
R=$GRAFT_REPO_ROOT; cd $R
for rep in 1 2; do
  for L in default qr1; do
    if [ $L = qr1 ]; then export LOAM_HIP_LIB=$R/loam_velodyne-1_amd/exp/qr1.so; else unset LOAM_HIP_LIB; fi
    echo "$L $(timeout -k 10 120 python tools/chain_bench.py 220)" || exit 1
    STEPS=30 BATCH=128 timeout -k 10 200 bash tools/ab_share.sh default | sed "s/^/$L /" || exit 1
  done
done
