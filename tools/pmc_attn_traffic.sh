#!/bin/bash
# HBM traffic of the bf16 attention kernels at the C2 shape (tools/attn_one.py): event timing,
# then separate FETCH_SIZE / WRITE_SIZE --pmc passes (VARIANTS: labels; the label "direct" sets
# RSYS_ATTN_DIRECT_STORE=1 for kernels that keep such an A/B switch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/attn_traffic
export TMPDIR=/tmp
for v in ${VARIANTS:-cur}; do
  if [ $v = direct ]; then export RSYS_ATTN_DIRECT_STORE=1; else unset RSYS_ATTN_DIRECT_STORE; fi
  timeout -k 10 120 python3 tools/attn_time.py 4096 50 0.1 bf16 > gpurun_out/attn_traffic/time_$v.log 2>&1
  rc=$?; echo "time $v rc=$rc: $(tail -1 gpurun_out/attn_traffic/time_$v.log)"; [ $rc -eq 0 ] || exit $rc
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace -d $ROOT/gpurun_out/attn_traffic/${v}_$ctr -o run --output-format csv -- python3 $ROOT/tools/attn_one.py 4096 50 0.1 bf16 ) > gpurun_out/attn_traffic/${v}_$ctr.log 2>&1
    rc=$?; echo "pmc $v $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
