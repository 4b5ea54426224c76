R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
Q="--cpu-sample 0 --latency-runs 0 --strong-leg 0 --stream-sweeps 0 --dense-batch 0 --steps 3 --warmup 1 --profile-steps 0"
cd /tmp
for v in 0 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ar_$v -o kt -- python3 $R/bench.py $Q --tune=od_win_mono=$v > $R/gpurun_out/ar_$v.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/ar_$v -name '*kernel_trace.csv' | head -1)
  echo od_win_mono=$v; python3 $R/tools/assoc_rounds.py $f
done
