R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
Q="--cpu-sample 0 --latency-runs 0 --strong-leg 0 --stream-sweeps 0 --dense-batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt128b -o kt -- python3 $R/bench.py --steps 10 --warmup 3 --batch 128 --global-batch 128 --profile-steps 0 $Q > $R/gpurun_out/kt128b.log 2>&1 || exit 1
python3 $R/tools/trace_timeline.py $R/gpurun_out/kt128b/kt_kernel_trace.csv --skip 3 --json $R/gpurun_out/kt128b_timeline.json > $R/gpurun_out/kt128b_timeline.txt
head -40 $R/gpurun_out/kt128b_timeline.txt
