#!/bin/bash
# round-5: the CE forward's rounded copies written by its finish kernel (bitwise
# test, A/B against the backward's own rounding launch, C2 timeline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16.py -k "ce" > gpurun_out/r5_s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_s_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "base= nouib=RSYS_CE_UIB=0 det=RSYS_DETERMINISTIC=1" "c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
