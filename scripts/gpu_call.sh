#!/bin/bash
# Round-4 call c: native partitioned BFS / SSSP / PageRank loops (ghost exchange).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04c
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py > gpurun_out/r04c/gpu_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|error" gpurun_out/r04c/gpu_tests.log | tail -12; tail -40 gpurun_out/r04c/gpu_tests.log | grep -v PASSED; exit $rc
