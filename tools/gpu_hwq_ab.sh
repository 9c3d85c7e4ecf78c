#!/bin/bash
# A/B of the hardware-queue count: the default line (C2 bf16 + C3 fp32/bf16) at GPU_MAX_HW_QUEUES
# = 4 (HIP's default, the box's setting) and 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/hwq_$q.log 2>&1 || exit 1
  python3 - "$q" <<'PY'
import json, sys
q = sys.argv[1]
s = open(f'gpurun_out/hwq_{q}.log').read()
d = json.loads(s[s.index('{"metric"'):].split('\n')[0])
print('hwq', q, 'c2', d['ms_per_step'], 'c3', d['extra']['c3']['ms_per_step'], 'c3bf16', d['extra']['c3_bf16']['ms_per_step'], flush=True)
PY
done
