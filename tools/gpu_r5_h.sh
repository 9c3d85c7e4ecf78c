#!/bin/bash
# round-5: the step-constant window in the id-order catch-up too: lazy-Adam, shard and DP tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_lazy_adam.py tests/test_gpu_shard.py tests/test_dist.py > gpurun_out/r5_h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_h_tests.log; exit $rc
