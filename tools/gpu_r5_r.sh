#!/bin/bash
# round-5: the CE forward's rounded copies (bitwise test, A/B), the deferred-reduce flush order
# (long jobs first vs queue order) and the wgrad row-split cap now that its partials are reduced in
# the shared flush; C2 bf16 and C3 fp32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16.py -k "ce" > gpurun_out/r5_r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_r_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "base= nouib=RSYS_CE_UIB=0 fifo=RSYS_DEFER_FIFO=1 cap256=RSYS_WGRAD_CAP=256 cap384=RSYS_WGRAD_CAP=384" "c2:bf16" || exit 1
REPS=1 bash tools/gpu_ab_env.sh "base= fifo=RSYS_DEFER_FIFO=1 cap256=RSYS_WGRAD_CAP=256" "c3:fp32" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
