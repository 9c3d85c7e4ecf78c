#!/bin/bash
# PMC passes (one --pmc set per run) over tools/lazy_bench.py; summaries per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmc_lazy
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $ROOT/gpurun_out/pmc_lazy/p$i -o run --output-format csv -- python3 $ROOT/tools/lazy_bench.py --iters 3 ${LB_ARGS} ) > gpurun_out/pmc_lazy/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
