#!/bin/bash
# Build libloam_hip.so from a committed revision's sources (default HEAD) into
# loam_velodyne-1_amd/exp/NAME.so, for an A/B against the working tree in one GPU call:
#   tools/build_ref_variant.sh NAME [REV] [-DFOO=1 ...]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; shift
rev=${1:-HEAD}; [ $# -gt 0 ] && shift
T=$(mktemp -d)
git -C "$ROOT" archive "$rev" loam_velodyne-1_amd/csrc include | tar -x -C "$T"
D="$ROOT/loam_velodyne-1_amd"
mkdir -p "$D/exp/$name.obj"
for f in sr.hip od.hip mp.hip engine.cpp bag.cpp msg.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function \
    -DLOAM_EXPERIMENT_BUILD "$@" -x hip -c "$T/loam_velodyne-1_amd/csrc/$f" -o "$D/exp/$name.obj/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$D/exp/$name.so" "$D/exp/$name.obj/"*.o -ldl
rm -rf "$D/exp/$name.obj" "$T"
echo "$D/exp/$name.so"
