mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_errors.py "tests/test_gpu_library.py::test_c2_step_through_torch_compile" "tests/test_gpu_workloads.py::test_c3_real_tables_lazy_matches_dense_adam" "tests/test_dist.py::test_eval_lookups_after_forward_row_sharded_two_ranks_one_gpu" > gpurun_out/r5_b_tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 60 python tools/capture_fork_repro.py chain_fresh > gpurun_out/r5_b_chain_fresh.log 2>&1; echo "chain_fresh rc=$?"
