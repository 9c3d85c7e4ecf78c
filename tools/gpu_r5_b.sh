#!/bin/bash
# round-5 checks: the new GPU tests, an A/B on C3 fp32 (uniform and Zipf ids: base, hot rows off,
# round-4 sort), then the captured RCCL step (last: it hung once; it dumps its stacks after 100 s)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_workloads.py::test_c3_capped_user_tower_own_stream_captured" \
  "tests/test_gpu_kernels.py::test_gather_hot_rows_bitwise" \
  "tests/test_gpu_library.py::test_c2_step_through_torch_compile" \
  "tests/test_gpu_workloads.py::test_c3_real_tables_lazy_matches_dense_adam" \
  "tests/test_gpu_workloads.py::test_c3_capped_matches_oracle" \
  "tests/test_dist.py::test_eval_lookups_after_forward_row_sharded_two_ranks_one_gpu" > gpurun_out/r5_b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5_b_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for z in "" "--zipf 1.05"; do
for v in base RSYS_NO_HOT_ROWS=1 RSYS_SORT_NO_RANK=1,RSYS_SORT_SMALL_TILES=1; do
  ( if [ "$v" != base ]; then for kv in ${v//,/ }; do export "$kv"; done; fi
    timeout -k 10 200 python bench.py --config c3 --dtype fp32 --no-cpu-baseline --extra= $z \
      > gpurun_out/r5_b_ab.json 2> gpurun_out/r5_b_ab.err ) || { tail -5 gpurun_out/r5_b_ab.err; exit 3; }
  python3 - "$rep" "$z" "$v" <<'PY' >> gpurun_out/r5_b_ab.txt
import json, sys
d = [json.loads(l)['bench_detail'] for l in open('gpurun_out/r5_b_ab.err') if l.startswith('{"bench_detail"')][-1]
k = d['kernel_ms_per_step']; g = d['gather_roofline']
print(sys.argv[1:], d['ms_per_step'], 'gather', g['rs_gather_fwd']['frac'], g['rs_gather_fwd']['ms_per_step'],
      'sort', k.get('rs_lookup_sort'), 'catchup', k.get('rs_sorted_catchup'), flush=True)
PY
  tail -1 gpurun_out/r5_b_ab.txt
done; done; done
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_errors.py > gpurun_out/r5_b_rccl.log 2>&1
rc=$?; echo "rccl rc=$rc"; tail -3 gpurun_out/r5_b_rccl.log; exit $rc
