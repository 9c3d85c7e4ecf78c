#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tower
( cd /tmp && DT=bf16 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace -d $ROOT/gpurun_out/pmc_tower/a -o run --output-format csv -- python3 $ROOT/tools/tower_phases.py ) > gpurun_out/pmc_tower/a.log 2>&1
echo "a rc=$?"
( cd /tmp && DT=bf16 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY --kernel-trace -d $ROOT/gpurun_out/pmc_tower/b -o run --output-format csv -- python3 $ROOT/tools/tower_phases.py ) > gpurun_out/pmc_tower/b.log 2>&1
echo "b rc=$?"
