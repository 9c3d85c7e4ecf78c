#!/bin/bash
# round-4 end profile set after the attention work: C2 bf16 and C3 fp32 kernel-trace summaries
# with FETCH_SIZE / WRITE_SIZE passes bracketing each line's dominant entry, then C2's one-step
# timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_prof_all.sh \
  "c2_bf16|auto|--config c2 --extra=" \
  "c3_fp32|auto|--config c3 --dtype fp32 --extra=" || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh || exit 1
