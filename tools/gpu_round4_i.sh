#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_library.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_i.log 2>&1; rc=$?; tail -2 gpurun_out/pt_i.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh "gs_on= gs_off=RSYS_GRAD_STREAMS=0" "c2:bf16"
