#!/bin/bash
# C2 step and token-GEMM time against the streaming GEMMs' row groups per workgroup
# (RSYS_STREAM_GROUPS; 12,800 groups at M = 204,800: 25 -> 512 workgroups, 50 -> 256)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sg
for g in ${GROUPS_LIST:-32 25 50 32}; do
  RSYS_STREAM_GROUPS=$g timeout -k 10 200 python bench.py --steps 30 --warmup 5 --extra c2 --no-cpu-baseline > gpurun_out/sg/g$g.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "g=$g rc=$rc"; exit $rc; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/sg/g$g.log') if l.startswith('{')][-1])
k=d['kernel_ms_per_step']
print('groups $g', d['ms_per_step'], 'tokens', k.get('rs_gemm_f32:tokens'), 'ffn_fwd', k.get('rs_ffn_fwd_bf16'), 'ln', k.get('rs_gemm_add_layernorm'))"
done
