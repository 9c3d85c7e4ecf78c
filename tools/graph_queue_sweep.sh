#!/bin/bash
# C3 bench under different hipGraph replay queue counts (DEBUG_HIP_FORCE_GRAPH_QUEUES) and
# GPU_MAX_HW_QUEUES settings: does the step's stream fork (item tower, per-table lookup chains)
# run in parallel inside the replayed graph? Usage: DT=bf16 bash tools/graph_queue_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DT=${DT:-bf16}
for q in default 2 4 8; do
  if [ "$q" = default ]; then
    timeout -k 10 200 python bench.py --config c3 --dtype "$DT" --no-cpu-baseline --extra= > gpurun_out/gq_$q.log 2>&1 || exit 1
  else
    DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 200 python bench.py --config c3 --dtype "$DT" --no-cpu-baseline --extra= > gpurun_out/gq_$q.log 2>&1 || exit 1
  fi
  python3 -c "
import json
s = open('gpurun_out/gq_$q.log').read()
i = s.index('{\"metric\"')
d = json.loads(s[i:].split('\n')[0])
print('$q', d['value'], d['ms_per_step'])"
done
