#!/bin/bash
# round-5: bf16 streaming-GEMM k order (64 contiguous bytes per row and load instruction): the
# bf16 tests, then the C2 line twice and its token-GEMM PMC traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16.py tests/test_gpu_parity.py > gpurun_out/r5_f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_f_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "kperm=" "c2:bf16 c5:bf16" || exit 1
grep -h '"rs_gemm_f32' gpurun_out/ab_kperm_c2_bf16.log | head -c 0
python3 - <<'PY'
import json
for cfg in ('c2_bf16', 'c5_bf16'):
    d = [json.loads(l)['bench_detail'] for l in open(f'gpurun_out/ab_kperm_{cfg}.log') if l.startswith('{"bench_detail"')][-1]
    k = d['kernel_ms_per_step']
    print(cfg, d['ms_per_step'], {x: k[x] for x in k if 'gemm' in x or 'ffn' in x}, d['roofline'].get('frac'), flush=True)
PY
