#!/bin/bash
# grouped-tower / hard-negative tests, then a short C5 line (bf16, 10 hard negatives)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hardneg.py tests/test_gpu_tower.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config c5 --hard-negatives 10 --steps 10 --warmup 3 --no-cpu-baseline --extra= > gpurun_out/b5.log 2>&1 || { tail -20 gpurun_out/b5.log; exit 4; }
tail -1 gpurun_out/b5.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('c5', d['ms_per_step'], d['value'], d['config']['host_issue_ms_per_step'])
print({k: v for k, v in list(d['kernel_ms_per_step'].items())[:14]})"
