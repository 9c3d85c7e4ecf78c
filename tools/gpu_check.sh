#!/bin/bash
# GPU round script: pytest -m gpu, smoke, short bench. Stops after any crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "STOP: rc=$1"; return 1;; esac; }
timeout -k 10 ${PYTEST_T:-900} python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 ${BENCH_T:-400} python bench.py --steps ${STEPS:-10} --warmup 3 --cpu-baseline-seconds ${CPU_S:-10} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
