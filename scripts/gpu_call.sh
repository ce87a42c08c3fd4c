#!/bin/bash
# Round-4 call b: the cross-rank push transpose of capped partition loads.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04b
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_gpu_assembly.py -k partition "tests/test_gpu_distributed.py" \
    "tests/test_gpu_fullsize.py::test_config5_rmat24_weighted_sssp_partitioned" \
    > gpurun_out/r04b/gpu_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|error" gpurun_out/r04b/gpu_tests.log | tail -30; tail -3 gpurun_out/r04b/gpu_tests.log; exit $rc
