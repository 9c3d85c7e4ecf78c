#!/bin/bash
# round-5: the clip partials' row kernel at 4 positions per group iteration: lazy-Adam tests
# (bitwise), then C3 fp32 and C5 bf16 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_lazy_adam.py tests/test_gpu_workloads.py -k "lazy or clip or c3" > gpurun_out/r5_j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_j_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "sq4=" "c3:fp32 c5:bf16"
