#!/bin/bash
# round-5: the one-hot MFMA table gradient, templated on its M tiles: gather tests, the isolated
# table-gradient timings under rocprofv3, A/B on C2 / C3, C2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "gather" > gpurun_out/r5_v_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_v_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/oh_time.py > gpurun_out/oh_time.log 2>&1
rc=$?; echo "oh rc=$rc"; [ $rc -eq 0 ] || exit $rc
cat gpurun_out/oh_time.log
REPS=2 bash tools/gpu_ab_env.sh "onehot= atomic=RSYS_NO_ONEHOT_GRAD=1" "c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
