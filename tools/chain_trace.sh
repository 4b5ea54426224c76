# Kernel trace of the config-3 device chain (tools/chain_bench.py) and its per-sweep timeline
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/chain_kt -o kt -- python3 $R/tools/chain_bench.py 220 > $R/gpurun_out/chain_kt.log 2>&1 || exit 1
f=$(find $R/gpurun_out/chain_kt -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_timeline.py $f --step-kernel k_sr_ring_count --skip 8 > $R/gpurun_out/chain_timeline.txt
head -45 $R/gpurun_out/chain_timeline.txt
