#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_ab_env.sh "base= tm64=RSYS_TOWER_TM=64 tm32=RSYS_TOWER_TM=32 prio=RSYS_USER_STREAM_PRIORITY=1" "c3:fp32 c2:bf16"
