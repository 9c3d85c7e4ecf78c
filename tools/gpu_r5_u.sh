#!/bin/bash
# round-5: the one-hot MFMA table gradient of tiny tables (gather_bwd_onehot_kernel): gather tests,
# C2 parity + library (deterministic-mode bitwise step), A/B against the atomic / slot kernels,
# C2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "gather" > gpurun_out/r5_u_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_u_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_library.py > gpurun_out/r5_u_tests2.log 2>&1
rc=$?; echo "tests2 rc=$rc"; tail -3 gpurun_out/r5_u_tests2.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "onehot= atomic=RSYS_NO_ONEHOT_GRAD=1" "c2:bf16 c3:fp32" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
