#!/bin/bash
# gather / attention / library / parity GPU tests, then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_library.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_f.log 2>&1; rc=$?; tail -3 gpurun_out/pt_f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 20 > gpurun_out/bench_full.log 2>&1; rc=$?
grep "^\[bench\]" gpurun_out/bench_full.log | tail -12
exit $rc
