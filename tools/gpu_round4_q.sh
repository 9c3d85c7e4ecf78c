#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -m gpu -x -q -k "gemm or stream or rowgemm or bf16" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_q.log 2>&1; rc=$?; tail -2 gpurun_out/pt_q.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for pr in prev=recommendsystemproject_amd/_lib/librsys_hip_prev.so new=recommendsystemproject_amd/_lib/librsys_hip.so; do
  lab=${pr%%=*}; path=${pr#*=}
  for cfg in c2 c5; do
  RSYS_LIB_PATH="$PWD/$path" timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --extra= > gpurun_out/abq_${lab}_${cfg}.log 2>&1 || { tail -5 gpurun_out/abq_${lab}_${cfg}.log; exit 1; }
  python3 - "$rep" "$lab" "$cfg" gpurun_out/abq_${lab}_${cfg}.log <<'PY' | tee -a gpurun_out/abq.txt
import json, sys
rep, lab, cfg, path = sys.argv[1:]
d = [json.loads(l) for l in open(path) if l.startswith('{"metric')][-1]
k = d['kernel_ms_per_step']
print(rep, cfg, lab, d['ms_per_step'], 'tokens', k.get('rs_gemm_f32:tokens'), 'frac', d['roofline']['frac'], flush=True)
PY
  done
done; done
