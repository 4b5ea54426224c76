#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root): bench line, rocprofv3 kernel trace +
# stats, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the same bench command.
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 300 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err && \
export TMPDIR=/tmp && cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o kt -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --stream-sweeps 0 > $R/gpurun_out/kt.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o f -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 0 --stream-sweeps 0 > $R/gpurun_out/fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o w -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 0 --stream-sweeps 0 > $R/gpurun_out/write.log 2>&1
