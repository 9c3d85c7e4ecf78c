#!/bin/bash
# Kernel-trace profile (rocprofv3 --kernel-trace --stats) of a short bench run, for
# tools/step_timeline.py. Usage: tools/gpu_trace.sh <config> [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
CFG=${1:-c2}; shift
OUT=gpurun_out/trace_$CFG
rm -rf $OUT && mkdir -p $OUT
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/trace -o run --output-format csv -- python3 $ROOT/bench.py --config $CFG --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline "$@" ) > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $OUT/trace.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $OUT > $OUT/summary.txt && python3 tools/step_timeline.py $OUT/trace > $OUT/timeline.txt
