#!/bin/bash
# the whole GPU suite (one pytest process), then the smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/suite.log 2>&1; rc=$?
tail -25 gpurun_out/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log
exit $rc
