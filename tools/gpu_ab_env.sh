#!/bin/bash
# env A/B of the bench line: bash tools/gpu_ab_env.sh "label=ENV1=v,ENV2=v label2=..." "config:dtype ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARS=$1; CFGS=${2:-c3:fp32}
for rep in $(seq 1 ${REPS:-2}); do
for cd in $CFGS; do
  cfg=${cd%%:*}; dt=${cd#*:}
  for v in $VARS; do
    lab=${v%%=*}; envs=${v#*=}; [ "$envs" = "$v" ] && envs=""
    ( for kv in ${envs//,/ }; do export "$kv"; done
      timeout -k 10 240 python bench.py --config $cfg --dtype $dt --no-cpu-baseline --extra= > gpurun_out/ab_${lab}_${cfg}_${dt}.log 2>&1 ) || { tail -5 gpurun_out/ab_${lab}_${cfg}_${dt}.log; exit 1; }
    python3 - "$rep" "$cfg" "$dt" "$lab" gpurun_out/ab_${lab}_${cfg}_${dt}.log <<'PY' | tee -a gpurun_out/ab_env.txt
import json, sys
rep, cfg, dt, lab, path = sys.argv[1:]
d = [json.loads(l)['bench_detail'] for l in open(path) if l.startswith('{"bench_detail"')][-1]
k = d['kernel_ms_per_step']
keys = ('rs_lookup_sort', 'rs_sorted_catchup', 'rs_gather_fwd', 'rs_gather_bwd', 'rs_segsum', 'rs_sorted_sqnorm_batch_dense', 'rs_sorted_adam_batch',
        'rs_sorted_adam_batch_dense', 'rs_tower_fwd', 'rs_tower_bwd')
print(rep, cfg, dt, lab, d['ms_per_step'], ' '.join(f'{x[3:]}={k.get(x, 0):.4f}' for x in keys), flush=True)
PY
  done
done; done
