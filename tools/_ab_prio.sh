#!/bin/bash
R=$GRAFT_REPO_ROOT; cd $R
STEPS=30 BATCH=128 bash tools/ab_share.sh default pipe_od_prio=1 default pipe_od_prio=1 || exit 1
STEPS=10 BATCH=1024 bash tools/ab_share.sh default pipe_od_prio=1 || exit 1
