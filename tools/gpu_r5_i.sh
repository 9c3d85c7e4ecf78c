#!/bin/bash
# round-5: the fused segment-sum fix with its level-2 tail blocks listed first: segsum tests, then
# C3 fp32 with the fused and the two-launch fix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_lazy_adam.py -k "segsum or sort" > gpurun_out/r5_i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_i_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "fused= two=RSYS_SEGSUM_TWO_FIX=1" "c3:fp32"
