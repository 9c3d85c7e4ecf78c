#!/bin/bash
# attention tests, attention timing (this build against the round-4 base build), the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -m gpu -x -q -k "attention or gather or pooled" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_attn.log 2>&1; rc=$?; tail -3 gpurun_out/pt_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_library.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_lib.log 2>&1; rc=$?; tail -3 gpurun_out/pt_lib.log; [ $rc -eq 0 ] || exit $rc
for lib in librsys_hip_r4base.so librsys_hip.so; do
  for shape in "4096 200" "4096 50"; do
    FULL=1 RSYS_LIB_PATH=$PWD/recommendsystemproject_amd/_lib/$lib timeout -k 10 120 python tools/attn_time.py $shape 0.1 bf16 > gpurun_out/at.txt 2>&1 || { cat gpurun_out/at.txt; exit 3; }
    echo "$lib $shape $(tail -1 gpurun_out/at.txt)" | tee -a gpurun_out/attn_ab.txt
  done
done
timeout -k 10 900 python bench.py --steps 20 > gpurun_out/bench_full.log 2>&1; rc=$?
tail -c 1500 gpurun_out/bench_full.log
exit $rc
