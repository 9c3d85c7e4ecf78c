#!/bin/bash
# round-5: fp32 fused CE occupancy variant (RSYS_CE_F32_OCC=1): its tests, microbench sweeps, then
# C3 fp32 with and without it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ce_f32.py > gpurun_out/r5_l_tests0.log 2>&1 && \
RSYS_CE_F32_OCC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ce_f32.py > gpurun_out/r5_l_tests1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5_l_tests0.log gpurun_out/r5_l_tests1.log; [ $rc -eq 0 ] || exit $rc
for v in "RSYS_CE_F32_OCC=0" "RSYS_CE_F32_OCC=1" "RSYS_CE_F32_OCC=1 RSYS_CE_SPLITS_FWD=32 RSYS_CE_SPLITS_BWD=16" \
         "RSYS_CE_F32_OCC=1 RSYS_CE_SPLITS_FWD=16 RSYS_CE_SPLITS_BWD=8" "RSYS_CE_F32_OCC=0 RSYS_CE_SPLITS_FWD=24 RSYS_CE_SPLITS_BWD=12"; do
  env $v CE_F32=1 timeout -k 10 120 python tools/ce_time.py 4096 128 50 >> gpurun_out/r5_l_ce.txt 2>&1 || exit 3
  echo "$v" >> gpurun_out/r5_l_ce.txt
done
cat gpurun_out/r5_l_ce.txt
REPS=2 bash tools/gpu_ab_env.sh "occ=RSYS_CE_F32_OCC=1 base=" "c3:fp32"
