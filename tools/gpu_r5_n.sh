#!/bin/bash
# round-5: the fused FFN backward's two LayerNorm partial reductions in one launch: bf16 / FFN
# tests, then the C2 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16.py tests/test_gpu_library.py > gpurun_out/r5_n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_n_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "red2=" "c2:bf16"
