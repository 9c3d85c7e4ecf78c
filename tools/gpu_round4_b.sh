#!/bin/bash
# tower tests + phases, the GPU suite, smoke, the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest tests/test_gpu_lazy_adam.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_sort.log 2>&1; rc=$?; tail -2 gpurun_out/pt_sort.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_tower.log 2>&1; rc=$?; tail -2 gpurun_out/pt_tower.log; [ $rc -eq 0 ] || exit $rc
DT=fp32 timeout -k 10 120 python tools/tower_phases.py > gpurun_out/phases_fp32.txt 2>&1 || exit 3
DT=bf16 timeout -k 10 120 python tools/tower_phases.py > gpurun_out/phases_bf16.txt 2>&1 || exit 3
cat gpurun_out/phases_fp32.txt gpurun_out/phases_bf16.txt | grep rs_
PYTEST_ARGS="--deselect tests/test_dist.py" bash tools/gpu_suite.sh || exit 5
bash tools/gpu_dist_check.sh || exit 6
timeout -k 10 900 python bench.py --steps 20 > gpurun_out/bench_full.log 2>&1; rc=$?
tail -c 1500 gpurun_out/bench_full.log
exit $rc
