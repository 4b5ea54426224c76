#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root), outputs under gpurun_out/prof_<TAG>:
#   bench.json      the default bench line
#   kt/             rocprofv3 --kernel-trace --stats of the batch-1024 workload
#   fetch/, write/  two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic per launch
#                   (tools/pmc_traffic.py -> traffic.json)
#   kt128/          kernel trace of the 8-GPU share (128 problems; tools/trace_timeline.py)
#   dkt/, dfetch/, dwrite/  the same for the config-5 batched leg alone (--dense-only)
#   ckt/            kernel trace of the config-3 device chain (tools/chain_bench.py, 220 sweeps)
R=$GRAFT_REPO_ROOT
TAG=${1:-r06}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
Q="--cpu-sample 0 --latency-runs 0 --strong-leg 0 --stream-sweeps 0 --dense-batch 0 --fed-leg 0"
D="--dense-only 1 --dense-batch 64 --cpu-sample 0"
cd $R && { [ "${BENCH:-1}" = 0 ] || timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; } && \
export TMPDIR=/tmp && cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --steps 5 --warmup 2 $Q > $O/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o f -- python3 $R/bench.py --steps 2 --warmup 1 --profile-steps 1 $Q > $O/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o w -- python3 $R/bench.py --steps 2 --warmup 1 --profile-steps 1 $Q > $O/write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt128 -o kt -- python3 $R/bench.py --steps 10 --warmup 3 --batch 128 --global-batch 128 --profile-steps 0 $Q > $O/kt128.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dkt -o kt -- python3 $R/bench.py --dense-steps 5 --profile-steps 0 $D > $O/dkt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/dfetch -o f -- python3 $R/bench.py --dense-steps 1 --profile-steps 1 $D > $O/dfetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/dwrite -o w -- python3 $R/bench.py --dense-steps 1 --profile-steps 1 $D > $O/dwrite.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ckt -o kt -- python3 $R/tools/chain_bench.py 220 > $O/ckt.log 2>&1
