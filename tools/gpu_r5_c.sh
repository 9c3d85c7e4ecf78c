cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_errors.py::test_rccl_captured_step_row_sharded_world_size_one" "tests/test_gpu_kernels.py::test_gather_hot_rows_bitwise" > gpurun_out/r5_c_rccl.log 2>&1
rc=$?; echo "rccl rc=$rc"; tail -3 gpurun_out/r5_c_rccl.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5_prof.sh
