#!/bin/bash
# round-5: the sequence input's dropout backward with the next row's loads in flight
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "seq_input or dropout" > gpurun_out/r5_ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_ab_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "base=" "c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
