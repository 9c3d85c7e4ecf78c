#!/bin/bash
# round-5 record, part 1: the whole GPU suite (one pytest process), the smoke, then the default
# bench line (stdout: the driver's JSON line; stderr: progress and the bench_detail record)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_final_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/r5_final_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_final_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r5_final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r5_final_bench.json 2> gpurun_out/r5_final_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r5_final_bench.json; exit $rc
