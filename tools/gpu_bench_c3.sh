#!/bin/bash
# C3 fp32 line with the bf16 and C2 extras; prints step time and host issue time per workload
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c3 --dtype fp32 --steps 30 --warmup 3 --no-cpu-baseline --extra ${EXTRA:-c3:bf16,c2} > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 4; }
tail -1 gpurun_out/b.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('c3', d['ms_per_step'], d['config']['host_issue_ms_per_step'])
for k, v in d.get('extra', {}).items():
    print(k, v.get('ms_per_step'), v.get('config', {}).get('host_issue_ms_per_step'), v.get('error', ''))"
