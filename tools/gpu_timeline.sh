#!/bin/bash
# one-step kernel timeline of a bench config (rocprofv3 kernel trace between the timed-region
# markers): CONFIG=c2|c3 DT=bf16|fp32 bash tools/gpu_timeline.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/tl_${CONFIG:-c2}_${DT:-bf16}
mkdir -p $OUT
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/trace -o run --output-format csv -- python3 $ROOT/bench.py --config ${CONFIG:-c2} --dtype ${DT:-bf16} --steps 10 --warmup 3 --no-cpu-baseline --prof-markers --extra= ) > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $OUT 10 ${CONFIG:-c2} > $OUT/summary.txt && python3 tools/step_timeline.py $OUT 4 > $OUT/timeline.txt; echo "post rc=$?"
