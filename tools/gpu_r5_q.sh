#!/bin/bash
# round-5: the deferred-reduce kernel with 16-byte loads: the bitwise deferred-vs-immediate test,
# then C2 with / without deferral and C2's one-step timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_prune.py > gpurun_out/r5_q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_q_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "defer= nodefer=RSYS_DEFER_REDUCE=0" "c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
