#!/bin/bash
# Round-4 A/B: committed library (prev) vs the rowgemm A-row ring (pf) vs ring + attention VALU
# trim + saved dropout keep bits (new, the in-tree build; nozb = new without the keep bits): full GPU suite on the new build, then C2 x2 and C5 x1 per library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_r.log 2>&1; rc=$?; tail -3 gpurun_out/pt_r.log; [ $rc -eq 0 ] || exit $rc
run() {  # rep label lib cfg
  RSYS_LIB_PATH="$PWD/$3" timeout -k 10 300 python bench.py --config $4 --no-cpu-baseline --extra= > gpurun_out/abr_$2_$4.log 2>&1 || { tail -5 gpurun_out/abr_$2_$4.log; exit 1; }
  python3 - "$1" "$2" "$4" gpurun_out/abr_$2_$4.log <<'PY' | tee -a gpurun_out/abr.txt
import json, sys
rep, lab, cfg, path = sys.argv[1:]
d = [json.loads(l) for l in open(path) if l.startswith('{"metric')][-1]
k = d['kernel_ms_per_step']
print(rep, cfg, lab, d['ms_per_step'], 'tokens', k.get('rs_gemm_f32:tokens'), 'attn_fwd', k.get('rs_attn_fwd'), 'attn_bwd', k.get('rs_attn_bwd'), flush=True)
PY
}
L=recommendsystemproject_amd/_lib
for rep in 1 2; do
  run $rep prev $L/librsys_hip_prev.so c2 || exit 1
  run $rep pf $L/librsys_hip_pf.so c2 || exit 1
  run $rep new $L/librsys_hip.so c2 || exit 1
  RSYS_ATTN_NO_ZBITS=1 run $rep nozb $L/librsys_hip.so c2 || exit 1
done
run 1 prev $L/librsys_hip_prev.so c5 || exit 1
run 1 new $L/librsys_hip.so c5 || exit 1
