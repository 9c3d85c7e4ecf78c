#!/bin/bash
# Same-box A/B of two source trees (each with its own built library): the bench line of every
# config from each tree, alternating, REPS repetitions.
#   bash tools/gpu_ab_tree.sh "old=_ab_old new=." "c3:fp32 c2:bf16"
# (_ab_old: `git archive <rev> | tar -x -C _ab_old` + make in its csrc; git-ignored)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
TREES=$1; CFGS=${2:-c3:fp32}
for rep in $(seq 1 ${REPS:-3}); do
for cd in $CFGS; do
  cfg=${cd%%:*}; dt=${cd#*:}
  for tv in $TREES; do
    lab=${tv%%=*}; dir=${tv#*=}
    log=$ROOT/gpurun_out/abt_${lab}_${cfg}_${dt}_${rep}.log
    ( cd $ROOT/$dir && timeout -k 10 240 python bench.py --config $cfg --dtype $dt --no-cpu-baseline --extra= ) > $log 2>&1 \
      || { tail -5 $log; exit 1; }
    python3 - "$rep" "$cfg" "$dt" "$lab" $log <<'PY' | tee -a $ROOT/gpurun_out/abt.txt
import json, sys
rep, cfg, dt, lab, path = sys.argv[1:]
d = [json.loads(l)['bench_detail'] for l in open(path) if l.startswith('{"bench_detail"')][-1]
k = d['kernel_ms_per_step']
top = sorted(k.items(), key=lambda kv: -kv[1])[:6]
print(rep, cfg, dt, lab, d['ms_per_step'], ' '.join(f'{a[3:]}={b:.4f}' for a, b in top), flush=True)
PY
  done
done; done
