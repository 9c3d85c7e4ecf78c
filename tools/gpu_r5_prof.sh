#!/bin/bash
# round-5 profile set: rocprofv3 kernel-trace summaries (C2 bf16, C3 fp32) with PMC traffic of each
# line's roofline entry (C2 / C5: the token GEMMs named explicitly -- 'auto' picks the entry that
# is largest in each --pmc pass, which differed between the FETCH and WRITE passes); PMC traffic of
# the gather at C3 (uniform and Zipf ids) and of C5's token GEMMs (bf16 and fp32, 10 hard
# negatives); C2's and C3's one-step timelines.
# Outputs: gpurun_out/prof_<tag>/ (traffic.json, summary.txt), gpurun_out/tl_<config>_<dtype>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_prof_all.sh \
  "c2_bf16|rs_gemm_f32:tokens|--config c2 --extra=" \
  "c3_fp32|auto|--config c3 --dtype fp32 --extra=" \
  "c3_fp32_gather|rs_gather_fwd|--config c3 --dtype fp32 --extra=|notrace" \
  "c3z_fp32_gather|rs_gather_fwd|--config c3 --dtype fp32 --zipf 1.05 --extra=|notrace" \
  "c5_bf16|rs_gemm_f32:tokens|--config c5 --hard-negatives 10 --extra=|notrace" \
  "c5_fp32|rs_gemm_f32:tokens|--config c5 --dtype fp32 --hard-negatives 10 --extra=|notrace" || exit 1
CONFIG=c3 DT=fp32 bash tools/gpu_timeline.sh || exit 1
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh
