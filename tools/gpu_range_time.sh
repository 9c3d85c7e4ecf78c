#!/bin/bash
# gather-backward tests, then rs_gather_bwd kernel times on C2's sequence-token tables
# (tools/range_time.py under rocprofv3 --kernel-trace), then a short C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_workloads.py -k "gather or golden or oracle or c2" > gpurun_out/t_gather.log 2>&1 || { tail -30 gpurun_out/t_gather.log; exit 1; }
tail -2 gpurun_out/t_gather.log
( cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/rt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/range_time.py ) > gpurun_out/rt.log 2>&1 || exit 1
python3 tools/range_trace.py gpurun_out/rt/run_kernel_trace.csv
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra= > gpurun_out/bench_c2.log 2>&1 || { tail -5 gpurun_out/bench_c2.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c2.log | head -1; grep -o '"rs_gather_bwd": [0-9.]*' gpurun_out/bench_c2.log
