#!/bin/bash
# A/B of library builds on the C3 bench: bash tools/ab_lib.sh "label=path label=path" [dtype ...]
# (path relative to the repository root; e.g. a variant built with make OUT=../_lib/variant.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
PAIRS=$1; shift; DTS=${*:-fp32}
for rep in 1 2; do
for dt in $DTS; do
for pr in $PAIRS; do
  lab=${pr%%=*}; path=${pr#*=}
  RSYS_LIB_PATH="$ROOT/$path" timeout -k 10 200 python bench.py --config c3 --dtype "$dt" --no-cpu-baseline --extra= > gpurun_out/ablib_${lab}_${dt}.log 2>&1 || exit 1
  python3 -c "
import json
s = open('gpurun_out/ablib_${lab}_${dt}.log').read()
i = s.index('{\"metric\"')
d = json.loads(s[i:].split('\n')[0])
k = d['kernel_ms_per_step']
print('$rep', '$dt', '$lab', d['value'], d['ms_per_step'], 'catchup', k.get('rs_sorted_catchup'), 'adam', k.get('rs_sorted_adam_batch'), flush=True)"
done; done; done
