#!/bin/bash
# round-5: the item tower's MLP held back until the user tower's first large-table sort is queued
# (RSYS_ITEM_HEAD_WAIT): workload / parity tests, then C3 fp32, C3 bf16 and C5 bf16 with it on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_workloads.py tests/test_gpu_parity.py tests/test_gpu_library.py > gpurun_out/r5_k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_k_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "wait= nowait=RSYS_ITEM_HEAD_WAIT=0" "c3:fp32 c3:bf16 c5:bf16"
