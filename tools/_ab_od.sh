#!/bin/bash
R=$GRAFT_REPO_ROOT; cd $R
STEPS=30 BATCH=128 bash tools/ab_share.sh default od_lm_mom_max=128 od_assoc_wg=32 od_assoc_wg=128 od_fused_max=0 default || exit 1
