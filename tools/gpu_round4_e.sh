#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/gbt -o run --output-format csv -- python3 $ROOT/tools/gather_bwd_time.py ) > gpurun_out/gbt.log 2>&1 || { tail -5 gpurun_out/gbt.log; exit 1; }
grep -v "^\s*$" gpurun_out/gbt.log | grep "us$"
ls gpurun_out/gbt
bash tools/gpu_ab_env.sh "new= sortML=RSYS_SORT_MULTILAUNCH=1 nont=RSYS_GATHER_NO_NT=1 oldgrad=RSYS_SLOT_GRAD=0,RSYS_RANGE_MIN_HITS=8 r3=RSYS_SORT_MULTILAUNCH=1,RSYS_GATHER_NO_NT=1,RSYS_SLOT_GRAD=0,RSYS_RANGE_MIN_HITS=8" "c3:fp32 c2:bf16"
