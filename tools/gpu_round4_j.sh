#!/bin/bash
# fused CE tests, CE timing with the bf16-streamed backward against RSYS_CE_STREAM_F32=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -m gpu -x -q -k "ce or loss" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_ce.log 2>&1; rc=$?; tail -2 gpurun_out/pt_ce.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -m gpu -x -q -k "attention" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_attn.log 2>&1; rc=$?; tail -2 gpurun_out/pt_attn.log; [ $rc -eq 0 ] || exit $rc
for lib in librsys_hip_prev.so librsys_hip.so; do
  FULL=1 RSYS_LIB_PATH=$PWD/recommendsystemproject_amd/_lib/$lib timeout -k 10 120 python tools/attn_time.py 4096 200 0.1 bf16 > gpurun_out/at.txt 2>&1 || { cat gpurun_out/at.txt; exit 3; }
  echo "$lib $(tail -1 gpurun_out/at.txt)" | tee -a gpurun_out/attn_ab.txt
done
for v in new f32; do
  if [ $v = f32 ]; then export RSYS_CE_STREAM_F32=1; fi
  timeout -k 10 120 python tools/ce_time.py 4096 128 > gpurun_out/ce_$v.txt 2>&1 || { cat gpurun_out/ce_$v.txt; exit 3; }
  echo "$v $(tail -1 gpurun_out/ce_$v.txt)"
  timeout -k 10 120 python tools/ce_time.py 4096 64 > gpurun_out/ce_${v}64.txt 2>&1 || { cat gpurun_out/ce_${v}64.txt; exit 3; }
  echo "$v D64 $(tail -1 gpurun_out/ce_${v}64.txt)"
done
unset RSYS_CE_STREAM_F32
REPS=1 bash tools/gpu_ab_env.sh "ce_b16= ce_f32=RSYS_CE_STREAM_F32=1 lk_off=RSYS_LOOKUP_STREAMS=0 tw_off=RSYS_TOWER_STREAMS=0" "c2:bf16 c3:bf16 c3:fp32"
