#!/bin/bash
# round-5: lookups-on-side modes (0 default, 2: user-tower lookup chains behind the item tower's
# forward on its stream) on C3 fp32 / C2 bf16, then one-step timelines of C2 bf16 and C3 fp32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
REPS=2 bash tools/gpu_ab_env.sh "m0= m2=RSYS_LOOKUPS_ON_SIDE=2" "c3:fp32 c2:bf16" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh || exit 1
CONFIG=c3 DT=fp32 bash tools/gpu_timeline.sh
