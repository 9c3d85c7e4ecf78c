#!/bin/bash
# C3 kernel-trace profile (rocprofv3 --kernel-trace --stats) of a short bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/c3prof
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/c3prof/trace -o run --output-format csv -- python3 $ROOT/bench.py --config c3 --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS} ) > gpurun_out/c3prof/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 gpurun_out/c3prof/trace.log
python3 tools/prof_summary.py gpurun_out/c3prof > gpurun_out/c3prof/summary.txt; echo "summary rc=$?"
