#!/bin/bash
# SQ counters for single rowgemm launches (tools/gemm_one.py): where do the wave cycles go?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for shape in "0 1 204800 256 64 0" "0 1 204800 256 64 19 0.1" "0 0 204800 256 64 8" "0 1 204800 64 256 0"; do
  i=$((i+1))
  ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d $ROOT/gpurun_out/pmc/s$i -o run --output-format csv -- python3 $ROOT/tools/gemm_one.py $shape ) > gpurun_out/pmc/s$i.log 2>&1
  rc=$?; echo "shape $i ($shape) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
