#!/bin/bash
# round-5: the deferred flush with several 256-column blocks per workgroup for short jobs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_prune.py tests/test_gpu_kernels.py -k "deferred or ranged or onehot or pruned" > gpurun_out/r5_ac_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_ac_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "base=" "c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
