#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench, then (PMC=1) HBM traffic of the dominant entry
# point: bench.py --pmc-bracket under separate FETCH_SIZE / WRITE_SIZE --pmc passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --prof-markers ${BENCH_ARGS}"
if [ -z "$NOTRACE" ]; then
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof/trace -o run --output-format csv -- python3 $ROOT/$B ) > gpurun_out/prof/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 gpurun_out/prof/trace.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PMC" ]; then
for ctr in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d $ROOT/gpurun_out/prof/pmc_$ctr -o run --output-format csv -- python3 $ROOT/bench.py --warmup 2 --pmc-bracket ${BRACKET:-auto} ${BENCH_ARGS} ) > gpurun_out/prof/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; tail -2 gpurun_out/prof/pmc_$ctr.log; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_traffic.py gpurun_out/prof gpurun_out/prof/pmc_FETCH_SIZE.log > gpurun_out/prof/traffic.json 2> gpurun_out/prof/traffic.err
echo "traffic rc=$?"; cat gpurun_out/prof/traffic.json | head -12
fi
[ -n "$NOTRACE" ] && exit 0
LABELS=$(python3 -c "import json,sys; l=[x for x in open(sys.argv[1]) if x.startswith('{\"metric')]; print(','.join(json.loads(l[-1]).get('prof_marker_order', [])))" gpurun_out/prof/trace.log 2>/dev/null)
python3 tools/prof_summary.py gpurun_out/prof ${STEPS:-10} "$LABELS" > gpurun_out/prof/summary.txt; echo "summary rc=$?"
