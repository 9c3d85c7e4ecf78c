#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -m gpu -x -q -k "attention" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_attn.log 2>&1; rc=$?; tail -2 gpurun_out/pt_attn.log; [ $rc -eq 0 ] || exit $rc
for lib in librsys_hip_prev.so librsys_hip.so; do
  for shape in "4096 200" "4096 100" "4096 65"; do
    FULL=1 RSYS_LIB_PATH=$PWD/recommendsystemproject_amd/_lib/$lib timeout -k 10 120 python tools/attn_time.py $shape 0.1 bf16 > gpurun_out/at.txt 2>&1 || { cat gpurun_out/at.txt; exit 3; }
    echo "$lib $shape $(tail -1 gpurun_out/at.txt)" | tee -a gpurun_out/attn_ab.txt
  done
done
timeout -k 10 400 python bench.py --config c5 --steps 10 --no-cpu-baseline --extra= > gpurun_out/bench_c5.log 2>&1; rc=$?
grep "^\[bench\]" gpurun_out/bench_c5.log | tail -3
exit $rc
