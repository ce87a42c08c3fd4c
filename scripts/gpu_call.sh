#!/bin/bash
# Round-4 call a: partition device assembly, split budget, partitioned weighted SSSP at RMAT-24,
# scale-27 one-GPU + world-2 partitioned tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04a
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_gpu_assembly.py tests/test_gpu_distributed.py "tests/test_gpu_parity.py::test_multi_source_split_budget_is_policy_only" \
    > gpurun_out/r04a/gpu_tests_1.log 2>&1 || { tail -40 gpurun_out/r04a/gpu_tests_1.log; exit 1; }
tail -5 gpurun_out/r04a/gpu_tests_1.log
TGO_TRACE=1 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
    tests/test_gpu_scale27.py "tests/test_gpu_fullsize.py::test_config5_rmat24_weighted_sssp_partitioned" \
    > gpurun_out/r04a/gpu_tests_2.log 2>&1
rc=$?; tail -30 gpurun_out/r04a/gpu_tests_2.log; exit $rc
