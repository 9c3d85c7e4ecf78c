#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=c2 DT=bf16 bash tools/gpu_timeline.sh && CONFIG=c3 DT=fp32 bash tools/gpu_timeline.sh
