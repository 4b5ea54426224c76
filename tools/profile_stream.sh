#!/bin/bash
# Kernel trace of the streaming node path (tools/stream_bench.py, configs 3 and 5)
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp && cd /tmp && \
STREAM_SWEEPS=60 STREAM_CPU_SWEEPS=10 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stream -o st -- python3 $R/tools/stream_bench.py > $R/gpurun_out/prof_stream.log 2>&1
