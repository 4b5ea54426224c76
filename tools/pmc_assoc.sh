#!/bin/bash
# SQ counters of the association kernel (diagnostic): one PMC pass, bench at batch 1024 (default
# tuning) -> gpurun_out/prof_assoc; summary: tools/pmc_summary.py
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp && cd /tmp && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --kernel-include-regex 'k_od_assoc|k_mp_nnfit|k_od_rows' --output-format csv -d $R/gpurun_out/prof_assoc -o sq -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 0 --stream-sweeps 0 --dense-batch 0 --fed-leg 0 > $R/gpurun_out/pmc_assoc.log 2>&1
