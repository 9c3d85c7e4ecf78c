#!/bin/bash
# SQ counter passes (instruction mix, wait buckets, MFMA busy) over a short bench run, one
# rocprofv3 --pmc pass per counter set (<= 8 SQ counters each), then tools/pmc_sq.py per kernel.
#   BENCH_ARGS="--config c2" bash tools/gpu_pmc_sq.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-sq}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES"
( cd /tmp && timeout -s KILL 60 rocprofv3 -L ) > $OUT/counters.txt 2>&1
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  for c in $P; do grep -q "$c" $OUT/counters.txt || { echo "counter $c not listed"; exit 3; }; done
  ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $P -d $OUT/pmc_$i -o run --output-format csv -- \
      python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --extra= ${BENCH_ARGS} ) > $OUT/pmc_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -2 $OUT/pmc_$i.log; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_sq.py $OUT > $OUT/sq_summary.jsonl; echo "summary rc=$?"; head -c 3000 $OUT/sq_summary.jsonl
