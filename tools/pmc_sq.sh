#!/bin/bash
# SQ counters of the L-M query kernels (diagnostic): one PMC pass, bench at batch 1024
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp && cd /tmp && \
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
  --kernel-include-regex 'k_mp_nnfit|k_od_assoc|k_sr_pick|k_sr_ringvg' --output-format csv -d $R/gpurun_out/prof_sq -o sq -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 0 --stream-sweeps 0 > $R/gpurun_out/sq.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
  --kernel-include-regex 'k_mp_nnfit|k_od_assoc|k_sr_pick|k_sr_ringvg' --output-format csv -d $R/gpurun_out/prof_tcc -o tcc -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-sample 0 --latency-runs 0 --strong-leg 0 --profile-steps 0 --stream-sweeps 0 > $R/gpurun_out/tcc.log 2>&1
