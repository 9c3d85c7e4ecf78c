#!/bin/bash
# round-5: the encoder's deferred flush and input-projection weight gradient on a side stream beside
# the sequence tables' gradients (ops.deferred_side): prune + parity tests, A/B, C2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_prune.py tests/test_gpu_parity.py > gpurun_out/r5_t_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_t_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "side= noside=RSYS_FLUSH_SIDE=0" "c2:bf16 c3:fp32" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
