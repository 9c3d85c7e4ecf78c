#!/bin/bash
# round-5: several tables' segment sums in one launch pair (rs_segsum_batch): lazy-Adam / workload /
# parity tests, A/B on C3 fp32 and C2, C3 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_lazy_adam.py tests/test_gpu_workloads.py tests/test_gpu_parity.py > gpurun_out/r5_ad_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_ad_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "batch= single=RSYS_SEGSUM_BATCH=0" "c3:fp32" || exit 1
CONFIG=c3 DT=fp32 bash tools/gpu_timeline.sh
