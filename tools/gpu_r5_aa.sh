#!/bin/bash
# round-5: the gradient norm's partials and the clip coefficient in one launch
# (rs_grad_sqnorm_clip_step): kernel / optimizer / parity tests, A/B, C2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_library.py tests/test_gpu_lazy_adam.py > gpurun_out/r5_aa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_aa_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "fused= split=RSYS_SQNORM_CLIP_FUSED=0" "c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
