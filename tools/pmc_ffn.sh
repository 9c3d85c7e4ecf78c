#!/bin/bash
# SQ counters of the fused FFN kernels (tools/ffn_one.py): where do the wave cycles go?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmcffn
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ffn_one.py 0.15 3 > gpurun_out/pmcffn/time_p15.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/ffn_one.py 0.0 3 > gpurun_out/pmcffn/time_p0.log 2>&1 || exit $?
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d $ROOT/gpurun_out/pmcffn/s$i -o run --output-format csv -- python3 $ROOT/tools/ffn_one.py 0.15 1 ) > gpurun_out/pmcffn/s$i.log 2>&1
  rc=$?; echo "set $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
