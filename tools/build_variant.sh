#!/bin/bash
# Build an experiment variant of libloam_hip.so with extra defines into loam_velodyne-1_amd/exp/:
#   tools/build_variant.sh NAME -DFOO=1 ...   -> loam_velodyne-1_amd/exp/NAME.so
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; shift
D="$ROOT/loam_velodyne-1_amd"
mkdir -p "$D/exp/$name.obj"
for f in sr.hip od.hip mp.hip engine.cpp bag.cpp msg.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function -DLOAM_EXPERIMENT_BUILD "$@" \
    -x hip -c "$D/csrc/$f" -o "$D/exp/$name.obj/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$D/exp/$name.so" "$D/exp/$name.obj/"*.o -ldl
rm -rf "$D/exp/$name.obj"
echo "$D/exp/$name.so"
