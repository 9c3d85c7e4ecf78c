#!/bin/bash
# round-5: the whole GPU suite (one pytest process), the smoke, then the C2 / C3 lines with the
# round-5 launch fusions on and off (RSYS_OPT_FUSE, RSYS_SEGSUM_TWO_FIX, RSYS_CE_SUM_LAUNCH,
# RSYS_LOOKUPS_ON_SIDE), two repetitions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_d_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r5_d_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_d_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r5_d_smoke.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "new= old=RSYS_OPT_FUSE=0,RSYS_SEGSUM_TWO_FIX=1,RSYS_CE_SUM_LAUNCH=1,RSYS_LOOKUPS_ON_SIDE=0" "c3:fp32 c2:bf16"
