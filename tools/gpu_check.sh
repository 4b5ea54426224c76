#!/bin/bash
# One GPU call's standard checks (run on the GPU box from the repo root): the -m gpu suite, then
# optionally an A/B of experiment libraries (AB="head other ..." at BATCH, see tools/ab_lib.sh) and
# the default bench line.  Outputs under gpurun_out/$TAG/.  Every GPU step under its own limit,
# chained: the first failure ends the call.
#   TAG=r06a AB="head diag" BENCH=1 bash tools/gpu_check.sh
R=$GRAFT_REPO_ROOT
TAG=${TAG:-chk}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
  tail -2 $O/gputest.log
fi
if [ -n "$AB" ]; then
  N=${N:-2} BATCH=${BATCH:-1024} STEPS=${STEPS:-10} timeout -k 10 900 bash tools/ab_lib.sh $AB > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
  cat $O/ab.txt
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python - $O/bench.json <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "frac", d["roofline"]["frac"], d["roofline"]["kernel"])
print("pipeline", d["pipeline"]["frac"], "survey", d["pipeline"]["survey_literal"]["frac"])
print("chain", d["single_stream"]["device_chain"]["ms_per_sweep"], d["single_stream"]["device_chain"].get("speedup_vs_cpu"))
print("share", d["weak"]["one_gpu_at_8gpu_share"])
print("dense", d["dense_batch"]["ms_per_step"], d["dense_batch"]["value"])
print(" ".join(f"{k}={v:.3f}" for k, v in sorted(d["kernel_ms_per_step"].items(), key=lambda kv: -kv[1])[:14]))
EOF
fi
if [ "${CHAIN:-0}" = 1 ]; then
  timeout -k 10 300 python tools/chain_split.py > $O/chain_split.txt 2>&1 || { tail -20 $O/chain_split.txt; exit 1; }
  cat $O/chain_split.txt
  TAGDIR=$O timeout -k 10 400 bash tools/chain_trace.sh > $O/chain_trace.txt 2>&1 || { tail -20 $O/chain_trace.txt; exit 1; }
  cp $R/gpurun_out/chain_timeline.txt $O/ 2>/dev/null
  head -60 $O/chain_trace.txt
fi
