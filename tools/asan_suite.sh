#!/bin/bash
# The CPU test suite (pytest -m "not gpu") under AddressSanitizer + UBSan ("Race
# detection / sanitizers").  Builds the sanitizer variants of the oracle (oracle/liboracle_asan.so),
# the engine's host code (libloam_hip_asan.so: engine, rosbag reader, message conventions; device
# code unchanged) and the sweep generator, preloads the shared clang ASan runtime into python and
# points the ctypes loaders at them.  CPU only (this container): no GPU sanitizer exists on the pool.
# Usage: tools/asan_suite.sh [pytest args...]   (log: profiles/r03/asan_suite.log when run by hand)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
make -C "$ROOT/oracle" asan >/dev/null
make -j8 -C "$ROOT/loam_velodyne-1_amd" asan >/dev/null
RT="$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n1)"
export LOAM_ORACLE_LIB="$ROOT/oracle/liboracle_asan.so"
export LOAM_HIP_LIB="$ROOT/loam_velodyne-1_amd/libloam_hip_asan.so"
export LOAM_SYNTH_LIB="$ROOT/loam_velodyne-1_amd/synth/libloam_synth_asan.so"
# leaks: python and the HIP runtime keep allocations to exit; everything else aborts the run
# reports go to files (pytest captures fd 2); printed below when the run fails
LOGDIR="$(mktemp -d /tmp/loam_asan.XXXXXX)"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0:log_path=$LOGDIR/asan"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:log_path=$LOGDIR/ubsan"
cd "$ROOT"
rc=0
LD_PRELOAD="$RT" python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@" || rc=$?
if compgen -G "$LOGDIR/*" >/dev/null; then echo "---- sanitizer reports ----"; cat "$LOGDIR"/*; rc=${rc:-1}; [ "$rc" = 0 ] && rc=1; fi
rm -rf "$LOGDIR"
exit $rc
