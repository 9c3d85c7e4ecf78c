#!/bin/bash
# Round-4 A/B: FFN grids for small row counts (librsys_hip_ffn.so) against the in-tree build:
# the FFN / pruned-layer / step tests on the variant, then C2 x2 and C5 x1 per library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=recommendsystemproject_amd/_lib
RSYS_LIB_PATH="$PWD/$L/librsys_hip_ffn.so" timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_prune.py tests/test_gpu_library.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_x.log 2>&1; rc=$?; tail -3 gpurun_out/pt_x.log; [ $rc -eq 0 ] || exit $rc
run() {  # rep label lib cfg
  RSYS_LIB_PATH="$PWD/$3" timeout -k 10 300 python bench.py --config $4 --no-cpu-baseline --extra= > gpurun_out/abx_$2_$4.log 2>&1 || { tail -5 gpurun_out/abx_$2_$4.log; exit 1; }
  python3 - "$1" "$2" "$4" gpurun_out/abx_$2_$4.log <<'PY' | tee -a gpurun_out/abx.txt
import json, sys
rep, lab, cfg, path = sys.argv[1:]
d = [json.loads(l) for l in open(path) if l.startswith('{"metric')][-1]
k = d['kernel_ms_per_step']
print(rep, cfg, lab, d['ms_per_step'], 'ffn_fwd', k.get('rs_ffn_fwd_bf16'), 'ffn_bwd', k.get('rs_ffn_bwd_ln2_bf16'), 'ffn_wgrad', k.get('rs_ffn_wgrad_bf16'), flush=True)
PY
}
for rep in 1 2; do
  run $rep base $L/librsys_hip.so c2 || exit 1
  run $rep ffn $L/librsys_hip_ffn.so c2 || exit 1
done
run 1 base $L/librsys_hip.so c5 || exit 1
run 1 ffn $L/librsys_hip_ffn.so c5 || exit 1
