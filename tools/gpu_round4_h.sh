#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
rm -rf gpurun_out/gbt
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/gbt -o run --output-format csv -- python3 $ROOT/tools/gather_bwd_time.py ) > gpurun_out/gbt.log 2>&1 || { tail -5 gpurun_out/gbt.log; exit 1; }
grep "us$" gpurun_out/gbt.log
bash tools/gpu_ab_env.sh "g1= g2=RSYS_BENCH_GRAPHS=2" "c2:bf16 c3:fp32"
