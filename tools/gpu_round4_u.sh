#!/bin/bash
# Round-4 A/B: attention-rows backward with LDS-staged whole-row stores (in-tree build) against the wsum_t
# build (prev): attention tests, then C2 and C5 x2 per library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_bf16.py tests/test_gpu_kernels.py -m gpu -x -q -k "attn or attention" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_u.log 2>&1; rc=$?; tail -3 gpurun_out/pt_u.log; [ $rc -eq 0 ] || exit $rc
run() {  # rep label lib cfg
  RSYS_LIB_PATH="$PWD/$3" timeout -k 10 300 python bench.py --config $4 --no-cpu-baseline --extra= > gpurun_out/abu_$2_$4.log 2>&1 || { tail -5 gpurun_out/abu_$2_$4.log; exit 1; }
  python3 - "$1" "$2" "$4" gpurun_out/abu_$2_$4.log <<'PY' | tee -a gpurun_out/abu.txt
import json, sys
rep, lab, cfg, path = sys.argv[1:]
d = [json.loads(l) for l in open(path) if l.startswith('{"metric')][-1]
k = d['kernel_ms_per_step']
print(rep, cfg, lab, d['ms_per_step'], 'attn_fwd', k.get('rs_attn_fwd'), 'attn_bwd', k.get('rs_attn_bwd'), 'rows', k.get('rs_attn_rows_fwd'), k.get('rs_attn_rows_bwd'), flush=True)
PY
}
L=recommendsystemproject_amd/_lib
for rep in 1 2; do
  for cfg in c2 c5; do
    run $rep prev $L/librsys_hip_prev.so $cfg || exit 1
    run $rep new $L/librsys_hip.so $cfg || exit 1
  done
done
