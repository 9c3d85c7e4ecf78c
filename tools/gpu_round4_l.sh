#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RSYS_ATTN_LONG_MIN=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -m gpu -x -q -k "attention" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_attn.log 2>&1; rc=$?; tail -2 gpurun_out/pt_attn.log; [ $rc -eq 0 ] || exit $rc
for v in 64 32; do
  FULL=1 RSYS_ATTN_LONG_MIN=$v timeout -k 10 120 python tools/attn_time.py 4096 50 0.1 bf16 > gpurun_out/at.txt 2>&1 || { cat gpurun_out/at.txt; exit 3; }
  echo "min$v full $(tail -1 gpurun_out/at.txt)" | tee -a gpurun_out/attn_ab.txt
  RSYS_ATTN_LONG_MIN=$v timeout -k 10 120 python tools/attn_time.py 4096 50 0.1 bf16 > gpurun_out/at.txt 2>&1 || { cat gpurun_out/at.txt; exit 3; }
  echo "min$v ragged $(tail -1 gpurun_out/at.txt)" | tee -a gpurun_out/attn_ab.txt
done
bash tools/gpu_ab_env.sh "short= long=RSYS_ATTN_LONG_MIN=32" "c2:bf16"
