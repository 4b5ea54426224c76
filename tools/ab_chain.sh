#!/bin/bash
# A/B of the chain: default vs launch choices, alternating N times; medians
R=$GRAFT_REPO_ROOT; cd $R
N=${N:-5}
: > gpurun_out/_chain_runs.txt
for rep in $(seq $N); do
  for C in "" "$@"; do
    r=$(timeout -k 10 120 python tools/chain_bench.py 220 $C) || exit 1
    echo "[$C] $r" >> gpurun_out/_chain_runs.txt
  done
done
python3 - <<'PY'
import re, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/_chain_runs.txt"):
    k = l[:l.index("]") + 1]
    d[k].append(float(re.search(r"([0-9.]+) ms per sweep", l).group(1)))
for k, v in d.items():
    v.sort()
    print(k, "median %.4f" % v[len(v) // 2], v)
PY
