#!/bin/bash
# round-4 profile set: kernel-trace summaries + HBM traffic (separate FETCH_SIZE / WRITE_SIZE
# --pmc passes) of C2 and C3 fp32, and the traffic of C3's gather and lazy-Adam chain entries
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_prof_all.sh \
  "c2_bf16|auto|--config c2 --extra=" \
  "c3_fp32|auto|--config c3 --dtype fp32 --extra=" \
  "c3_fp32_gather|rs_gather_fwd|--config c3 --dtype fp32 --extra=|1" \
  "c3_fp32_sorted_catchup|rs_sorted_catchup|--config c3 --dtype fp32 --extra=|1" \
  "c3_fp32_sorted_adam_batch|rs_sorted_adam_batch|--config c3 --dtype fp32 --extra=|1"
