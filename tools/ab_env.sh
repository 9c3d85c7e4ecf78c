#!/bin/bash
# A/B of one environment switch on the C3 bench: bash tools/ab_env.sh VAR "v0 v1" [dtype ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1; VALS=$2; shift 2; DTS=${*:-fp32 bf16}
for rep in 1 2; do
for dt in $DTS; do
for v in $VALS; do
  env "$VAR=$v" timeout -k 10 200 python bench.py --config c3 --dtype "$dt" --no-cpu-baseline --extra= > gpurun_out/ab_${VAR}_${v}_${dt}.log 2>&1 || exit 1
  python3 -c "
import json
s = open('gpurun_out/ab_${VAR}_${v}_${dt}.log').read()
i = s.index('{\"metric\"')
d = json.loads(s[i:].split('\n')[0])
print('$rep', '$dt', '$VAR=$v', d['value'], d['ms_per_step'], flush=True)"
done; done; done
