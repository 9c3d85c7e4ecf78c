#!/bin/bash
# Round-4 A/B: the dense clip's norm / coefficient formed by the sqnorm launch's last workgroup
# (rs_grad_sqnorm_coef) against the two launches (RSYS_CLIP_TWO_LAUNCHES=1): the full GPU suite,
# then C2 x2 and C5 x1 per variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_z.log 2>&1; rc=$?; tail -3 gpurun_out/pt_z.log; [ $rc -eq 0 ] || exit $rc
run() {  # rep label cfg (env from the caller)
  timeout -k 10 300 python bench.py --config $3 --no-cpu-baseline --extra= > gpurun_out/abz_$2_$3.log 2>&1 || { tail -5 gpurun_out/abz_$2_$3.log; exit 1; }
  python3 - "$1" "$2" "$3" gpurun_out/abz_$2_$3.log <<'PY' | tee -a gpurun_out/abz.txt
import json, sys
rep, lab, cfg, path = sys.argv[1:]
d = [json.loads(l) for l in open(path) if l.startswith('{"metric')][-1]
k = d['kernel_ms_per_step']
print(rep, cfg, lab, d['ms_per_step'], 'sqnorm', k.get('rs_grad_sqnorm'), k.get('rs_grad_sqnorm_coef'), 'clip', k.get('rs_clip_coef_step'), flush=True)
PY
}
for rep in 1 2; do
  RSYS_CLIP_TWO_LAUNCHES=1 run $rep two c2 || exit 1
  run $rep one c2 || exit 1
done
RSYS_CLIP_TWO_LAUNCHES=1 run 1 two c5 || exit 1
run 1 one c5 || exit 1
