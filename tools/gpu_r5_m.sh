#!/bin/bash
# round-5: the pruned last layer's out-proj + residual + LayerNorm through the fused bf16 kernel at
# B rows: prune / bf16 tests, then C2 with it on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_prune.py tests/test_gpu_bf16.py > gpurun_out/r5_m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_m_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "lnf= lnu=RSYS_SMALL_LN_UNFUSED=1" "c2:bf16"
python3 - <<'PY'
import json
for lab in ('lnf', 'lnu'):
    d = [json.loads(l)['bench_detail'] for l in open(f'gpurun_out/ab_{lab}_c2_bf16.log') if l.startswith('{"bench_detail"')][-1]
    k = d['kernel_ms_per_step']
    print(lab, d['ms_per_step'], {x: k[x] for x in k if 'layernorm' in x or 'gemm' in x})
PY
