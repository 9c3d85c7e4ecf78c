#!/bin/bash
# the distributed GPU tests, then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS="tests/test_dist.py -k sharded_with_max_pooled" bash tools/gpu_dist_check.sh || exit 6
timeout -k 10 900 python bench.py --steps 20 > gpurun_out/bench_full.log 2>&1; rc=$?
tail -c 1500 gpurun_out/bench_full.log
exit $rc
