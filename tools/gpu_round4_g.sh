#!/bin/bash
# attention tests + timing of this build, then the encoder weight-gradient stream A/B at C2 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -m gpu -x -q -k "attention" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_attn.log 2>&1; rc=$?; tail -2 gpurun_out/pt_attn.log; [ $rc -eq 0 ] || exit $rc
for shape in "4096 200" "4096 50"; do
  FULL=1 timeout -k 10 120 python tools/attn_time.py $shape 0.1 bf16 > gpurun_out/at.txt 2>&1 || { cat gpurun_out/at.txt; exit 3; }
  echo "new $shape $(tail -1 gpurun_out/at.txt)" | tee -a gpurun_out/attn_ab.txt
done
bash tools/gpu_ab_env.sh "wg_on= wg_off=RSYS_WGRAD_STREAM=0" "c2:bf16"
