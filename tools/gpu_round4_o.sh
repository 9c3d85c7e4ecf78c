#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_o.log 2>&1; rc=$?; tail -2 gpurun_out/pt_o.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh "base= tm32=RSYS_TOWER_TM=32" "c3:fp32 c3:bf16 c2:bf16"
