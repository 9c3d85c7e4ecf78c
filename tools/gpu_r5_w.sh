#!/bin/bash
# round-5: the one-hot table gradient at C5's 819,200 history tokens (rows per wave capped at 128)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "onehot" > gpurun_out/r5_w_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_w_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "onehot= atomic=RSYS_NO_ONEHOT_GRAD=1" "c5:bf16" || exit 1
