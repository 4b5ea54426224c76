#!/bin/bash
# Copy the judged summaries of a tools/profile.sh run (gpurun_out/prof_TAG) into profiles/DEST:
#   tools/profile_post.sh TAG DEST
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
S=$R/gpurun_out/prof_$1
D=$R/profiles/$2
mkdir -p $D
[ -f $S/bench.json ] && cp $S/bench.json $D/bench.json
cp $S/kt/kt_kernel_stats.csv $D/kernel_stats_batch1024.csv
cp $S/kt128/kt_kernel_stats.csv $D/kernel_stats_share128.csv
cp $S/dkt/kt_kernel_stats.csv $D/kernel_stats_config5_batch64.csv
python3 $R/tools/pmc_traffic.py $S/fetch/f_counter_collection.csv $S/write/w_counter_collection.csv $R/profiles/traffic.json $D/pmc_traffic.csv
python3 $R/tools/pmc_traffic.py $S/dfetch/f_counter_collection.csv $S/dwrite/w_counter_collection.csv $R/profiles/traffic_config5.json $D/pmc_traffic_config5.csv
python3 $R/tools/trace_timeline.py $S/kt/kt_kernel_trace.csv --step-kernel k_sr_ring_fused --skip 2 > $D/timeline_batch1024.txt
python3 $R/tools/trace_timeline.py $S/kt128/kt_kernel_trace.csv --step-kernel k_sr_ring_fused --skip 3 > $D/timeline_share128.txt
python3 $R/tools/trace_timeline.py $S/dkt/kt_kernel_trace.csv --step-kernel k_sr_ring_fused --skip 2 > $D/timeline_config5_batch64.txt
if [ -d $S/ckt ]; then
  cp $S/ckt/kt_kernel_stats.csv $D/kernel_stats_chain220.csv
  python3 $R/tools/trace_timeline.py $S/ckt/kt_kernel_trace.csv --step-kernel k_sr_ring_count --skip 8 > $D/timeline_chain220.txt
fi
echo "$D"
