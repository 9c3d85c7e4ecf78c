#!/bin/bash
# HBM traffic of C3's lazy-Adam chain entries after a full cycle of the resident batches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_prof_all.sh \
  "c3_fp32_sorted_catchup|rs_sorted_catchup|--config c3 --dtype fp32 --extra=|1" \
  "c3_fp32_sorted_adam_batch|rs_sorted_adam_batch|--config c3 --dtype fp32 --extra=|1" \
  "c3_fp32_gather|rs_gather_fwd|--config c3 --dtype fp32 --extra=|1"
