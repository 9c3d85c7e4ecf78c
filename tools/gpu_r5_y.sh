#!/bin/bash
# round-5: the backward's scatter, small-table and dense work in one launch (gather_bwd_fused_kernel):
# kernel / library / parity tests, A/B against three launches, C2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_library.py tests/test_gpu_parity.py tests/test_gpu_tower.py > gpurun_out/r5_y_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_y_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "fused= split=RSYS_GATHER_BWD_SPLIT=1" "c2:bf16 c3:fp32" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
