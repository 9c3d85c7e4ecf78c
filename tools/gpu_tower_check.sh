set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_tower.log 2>&1; rc=$?; tail -3 gpurun_out/pt_tower.log; [ $rc -eq 0 ] || exit $rc
DT=fp32 timeout -k 10 120 python tools/tower_phases.py > gpurun_out/phases_fp32.txt 2>&1 || exit 3
DT=bf16 timeout -k 10 120 python tools/tower_phases.py > gpurun_out/phases_bf16.txt 2>&1 || exit 3
cat gpurun_out/phases_fp32.txt gpurun_out/phases_bf16.txt
timeout -k 10 300 python bench.py --config c3 --dtype fp32 --steps 20 --warmup 3 --no-cpu-baseline --extra c3:bf16 > gpurun_out/bench_c3.log 2>&1 || exit 4
tail -1 gpurun_out/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 fp32', d['ms_per_step'], {k:v for k,v in d['kernel_ms_per_step'].items() if 'tower' in k}); e=d['extra']; [print(k, v['ms_per_step'], {kk:vv for kk,vv in v['kernel_ms_per_step'].items() if 'tower' in kk}) for k,v in e.items()]"
