R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --runtime-trace --output-format csv -d $R/gpurun_out/chain_rt -o rt -- python3 $R/tools/chain_bench.py 80 > $R/gpurun_out/chain_rt.log 2>&1 || exit 1
ls -la $R/gpurun_out/chain_rt/ | head
