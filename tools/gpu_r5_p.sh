#!/bin/bash
# round-5: the pruned last layer's residual rows read in place by the fused LN kernel
# (RSYS_LN_ROWS): prune / bf16 / parity / library tests, then C2 with it on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_prune.py tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_library.py > gpurun_out/r5_p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_p_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "rows= gath=RSYS_LN_ROWS=0" "c2:bf16"
