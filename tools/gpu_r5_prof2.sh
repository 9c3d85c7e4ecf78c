#!/bin/bash
# round-5 end profile set: rocprofv3 kernel-trace summaries and PMC traffic of the roofline entry
# (C2 bf16 token GEMMs, C3 fp32 auto), C3's one-step timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_prof_all.sh \
  "c2_bf16|rs_gemm_f32:tokens|--config c2 --extra=" \
  "c3_fp32|auto|--config c3 --dtype fp32 --extra=" || exit 1
CONFIG=c3 DT=fp32 bash tools/gpu_timeline.sh
