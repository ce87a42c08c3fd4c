#!/bin/bash
# Deferred device decode + partitioned changes: decode/scan/distributed GPU tests, plain bench
# (config2 load: device vs host decode), partitioned world-1 profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02ah
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_scan.py tests/test_gpu_distributed.py \
    tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02ah/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02ah/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/r02ah/bench.json 2> gpurun_out/r02ah/bench.err
rc=$?; echo "bench exit $rc"; tail -2 gpurun_out/r02ah/bench.err; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_part_prof.sh
