#!/bin/bash
# data-parallel GPU tests (gloo ranks sharing the one GPU): W = 2 parity, row sharding, C4 at W = 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests/test_dist.py} -m gpu -x -v --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/dist.log 2>&1; rc=$?
tail -15 gpurun_out/dist.log
exit $rc
