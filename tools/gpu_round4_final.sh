#!/bin/bash
# the full GPU suite, smoke, the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_suite.sh || exit 5
timeout -k 10 900 python bench.py --steps 20 > gpurun_out/bench_full.log 2>&1; rc=$?
grep "^\[bench\]" gpurun_out/bench_full.log | tail -12
exit $rc
