#!/bin/bash
# Batch (config 4) A/B of experiment builds: for each library given, a short bench line with the
# per-kernel ms/step (LOAM_HIP_LIB selects the library).  Outputs gpurun_out/exp_<name>.json
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B=${BATCH:-1024}
for L in "$@"; do
  n=$(basename $L .so)_$B
  LOAM_HIP_LIB=$R/$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --latency-runs 0 \
    --batch $B --global-batch $B \
    --strong-leg 0 --stream-sweeps 0 ${TUNE:+--tune=$TUNE} > gpurun_out/exp_$n.json 2> gpurun_out/exp_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp_$n.json'));k=d['kernel_ms_per_step'];print('$n',round(d['ms_per_step'],3),'nnfit',k.get('k_mp_nnfit'),'assoc',k.get('k_od_assoc'),'vgs',k.get('vg_stack'),'vgc',k.get('vg_cubes'),'rows',k.get('k_od_rows'),'iter',k.get('k_mp_iter'),'sel',k.get('k_sr_select'),'hl',k.get('k_hash_build_last'),'hm',k.get('k_hash_build_map'),'ins',k.get('k_mp_insert'),'cmp',k.get('k_mp_compact'),'reg',k.get('k_mp_register'),'end',k.get('k_od_end'),'endseed',k.get('k_od_end_seed'))"
done
