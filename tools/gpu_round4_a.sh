#!/bin/bash
# round 4: tower phases (fp32 / bf16), the item tower's capture order A/B, then the DP tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DT=fp32 timeout -k 10 120 python tools/tower_phases.py > gpurun_out/phases_fp32.txt 2>&1 || exit 3
DT=bf16 timeout -k 10 120 python tools/tower_phases.py > gpurun_out/phases_bf16.txt 2>&1 || exit 3
echo phases done
for o in first last first last; do
  RSYS_ITEM_ORDER=$o timeout -k 10 240 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/order_$o.log 2>&1 || exit 4
  python3 - "$o" <<'PY'
import json, sys
o = sys.argv[1]
s = open(f'gpurun_out/order_{o}.log').read()
d = json.loads(s[s.index('{"metric"'):].split('\n')[0])
print('item order', o, 'c2', d['ms_per_step'], 'c3', d['extra']['c3']['ms_per_step'], 'c3bf16', d['extra']['c3_bf16']['ms_per_step'], flush=True)
PY
done
bash tools/gpu_dist_check.sh
