#!/bin/bash
# A/B of the config-3 device chain across libraries (loam_velodyne-1_amd/exp/NAME.so, see
# tools/build_ref_variant.sh) against the working tree, alternating 5 times; medians:
#   tools/ab_chain_lib.sh base [other ...]
R=$GRAFT_REPO_ROOT; cd $R
: > gpurun_out/_chain_lib.txt
for rep in 1 2 3 4 5; do
  for L in tree "$@"; do
    if [ $L = tree ]; then unset LOAM_HIP_LIB; else export LOAM_HIP_LIB=$R/loam_velodyne-1_amd/exp/$L.so; fi
    r=$(timeout -k 10 120 python tools/chain_bench.py 220) || exit 1
    echo "[$L] $r" >> gpurun_out/_chain_lib.txt
  done
done
python3 - <<'PY'
import re, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/_chain_lib.txt"):
    k = l[:l.index("]") + 1]
    d[k].append(float(re.search(r"([0-9.]+) ms per sweep", l).group(1)))
for k, v in d.items():
    v.sort()
    print(k, "median %.4f" % v[len(v) // 2], v)
PY
