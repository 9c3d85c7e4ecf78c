#!/bin/bash
# lazy-table / sort / shard / tower tests, then the C3 line (fp32 + bf16 extra)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_lazy_adam.py tests/test_gpu_shard.py tests/test_gpu_tower.py tests/test_gpu_workloads.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
EXTRA=c3:bf16 bash tools/gpu_bench_c3.sh
