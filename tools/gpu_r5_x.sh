#!/bin/bash
# round-5: dense-feature backward with shuffled row-lane sums, no output-gradient copy before the
# fused bf16 last layer: kernel / prune / parity tests, C2 bench x2, C2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_prune.py tests/test_gpu_parity.py > gpurun_out/r5_x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_x_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "base=" "c2:bf16 c3:fp32" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
