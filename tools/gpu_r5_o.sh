#!/bin/bash
# round-5: the encoder backward's parameter-gradient reductions deferred to one launch
# (RSYS_DEFER_REDUCE): encoder / bf16 / library / parity tests, then C2 and C5 bf16 on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_library.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_prune.py \
  tests/test_gpu_workloads.py > gpurun_out/r5_o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_o_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "defer= nodefer=RSYS_DEFER_REDUCE=0" "c2:bf16 c5:bf16"
