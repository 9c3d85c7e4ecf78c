#!/bin/bash
# quick GPU loop: tower / parity / bf16 tests, tower phases, C3 fp32 + bf16 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_tower.py tests/test_gpu_parity.py tests/test_gpu_bf16.py} -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
DT=fp32 timeout -k 10 120 python tools/tower_phases.py > gpurun_out/phases.txt 2>&1 || exit 3
grep rs_ gpurun_out/phases.txt
timeout -k 10 200 python bench.py --config c3 --dtype fp32 --steps 30 --warmup 3 --no-cpu-baseline --extra c3:bf16 > gpurun_out/b.log 2>&1 || exit 4
tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['extra']['c3_bf16']['ms_per_step'], d['kernel_ms_per_step'])"
