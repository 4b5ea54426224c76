#!/bin/bash
# SQ counters of one kernel family (diagnostic), two PMC passes over a 1-step bench at batch 1024.
#   tools/pmc_kernel.sh <kernel-regex> <tag>
R=$GRAFT_REPO_ROOT
RX=${1:-k_sr_select}
TAG=${2:-k}
shift 2 2>/dev/null
EXTRA=("$@")  # further bench.py arguments (e.g. --tune=mp_fused_max=0 --batch 128 --global-batch 128)
export TMPDIR=/tmp && cd /tmp && \
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS \
  --kernel-include-regex "$RX" --output-format csv -d $R/gpurun_out/pmc_${TAG}_a -o a -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 0 --stream-sweeps 0 --dense-batch 0 "${EXTRA[@]}" > $R/gpurun_out/pmc_${TAG}_a.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES \
  --kernel-include-regex "$RX" --output-format csv -d $R/gpurun_out/pmc_${TAG}_b -o b -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 0 --stream-sweeps 0 --dense-batch 0 "${EXTRA[@]}" > $R/gpurun_out/pmc_${TAG}_b.log 2>&1
