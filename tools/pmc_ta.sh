#!/bin/bash
# Texture-address / L1 / L2 counters of one kernel family (diagnostic), one PMC pass over a 1-step
# bench at batch 1024.   tools/pmc_ta.sh <kernel-regex> <tag>
R=$GRAFT_REPO_ROOT
RX=${1:-k_mp_nnfit}
TAG=${2:-k}
shift 2 2>/dev/null
EXTRA=("$@")  # further bench.py arguments (e.g. --tune=mp_fused_max=0 --batch 128 --global-batch 128)
export TMPDIR=/tmp && cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
  --kernel-include-regex "$RX" --output-format csv -d $R/gpurun_out/pmc_${TAG}_ta -o ta -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --profile-steps 0 --stream-sweeps 0 --latency-runs 0 --strong-leg 0 --dense-batch 0 "${EXTRA[@]}" > $R/gpurun_out/pmc_${TAG}_ta.log 2>&1
