#!/bin/bash
# Round-4 call o: Long / Double weight keys (generic tests), codec / rows / write-back tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_generic.py tests/test_gpu_parity.py tests/test_gpu_decode.py tests/test_gpu_writeback.py \
    > gpurun_out/r04o/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04o/tests.log | tail -12; exit $rc
