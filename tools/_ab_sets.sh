#!/bin/bash
R=$GRAFT_REPO_ROOT; cd $R
STEPS=30 BATCH=128 bash tools/ab_share.sh default pipe_sr_sets=2 default pipe_sr_sets=2 || exit 1
STEPS=10 BATCH=1024 bash tools/ab_share.sh default pipe_sr_sets=2 || exit 1
LOAM_HIP_LIB=$R/loam_velodyne-1_amd/exp/ptrace.so timeout -k 10 120 python tools/host_enqueue.py 128 16 > gpurun_out/pt128b.txt 2>&1
