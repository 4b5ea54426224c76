#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root): the default bench line, a rocprofv3
# kernel trace + stats of the same workload, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# for the HBM traffic per launch (tools/pmc_traffic.py).  Outputs under gpurun_out/prof_<TAG>.
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd $R && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && \
export TMPDIR=/tmp && cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --stream-sweeps 0 > $O/kt.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o f -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 1 --stream-sweeps 0 > $O/fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o w -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 1 --stream-sweeps 0 > $O/write.log 2>&1
