#!/bin/bash
# A/B of the chain: default vs launch choices, alternating
R=$GRAFT_REPO_ROOT; cd $R
for rep in 1 2; do
  for C in "" "mp_defer=0"; do
    echo "$(timeout -k 10 120 python tools/chain_bench.py 220 $C)" || exit 1
  done
done
