#!/bin/bash
# round-5: the ranged and one-hot table gradients in one launch (gather_bwd_tail_kernel): kernel /
# parity tests, A/B against separate launches, C2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_prune.py > gpurun_out/r5_z_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_z_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "fused= split=RSYS_GATHER_BWD_SPLIT=1" "c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
