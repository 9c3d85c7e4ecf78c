#!/bin/bash
# CE / workload tests, then a C3 bench (fp32 with the bf16 extra) -- GPU round helper
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ce_f32.py tests/test_gpu_workloads.py tests/test_gpu_library.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_ce.log 2>&1; rc=$?; tail -3 gpurun_out/pt_ce.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --dtype fp32 --steps 20 --warmup 3 --no-cpu-baseline --extra c3:bf16 > gpurun_out/bench_c3.log 2>&1 || exit 4
tail -1 gpurun_out/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 fp32', d['ms_per_step'], d['batch_dot_roofline'], {k:v for k,v in d['kernel_ms_per_step'].items() if 'tower' in k or 'ce' in k}); e=d['extra']; [print(k, v['ms_per_step']) for k,v in e.items()]"
