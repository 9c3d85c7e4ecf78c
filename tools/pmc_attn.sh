#!/bin/bash
# SQ counters for the attention kernels at the C2 shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmc_attn
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d $ROOT/gpurun_out/pmc_attn/a -o run --output-format csv -- python3 $ROOT/tools/attn_one.py 4096 50 0.1 ${DTYPE:-fp32} ) > gpurun_out/pmc_attn/a.log 2>&1
rc=$?; echo "pass a rc=$rc"; [ $rc -eq 0 ] || exit $rc
( cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-trace -d $ROOT/gpurun_out/pmc_attn/b -o run --output-format csv -- python3 $ROOT/tools/attn_one.py 4096 50 0.1 ${DTYPE:-fp32} ) > gpurun_out/pmc_attn/b.log 2>&1
rc=$?; echo "pass b rc=$rc"; tail -3 gpurun_out/pmc_attn/b.log; exit $rc
