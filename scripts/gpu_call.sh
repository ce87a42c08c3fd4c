#!/bin/bash
# Round-4 call c: native partitioned BFS / SSSP / PageRank loops (ghost exchange), device RMAT partition.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04c
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py > gpurun_out/r04c/gpu_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|error" gpurun_out/r04c/gpu_tests.log | tail -6; tail -40 gpurun_out/r04c/gpu_tests.log | grep -v PASSED
[ $rc -eq 0 ] || exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 600 python3 bench.py --partitioned --steps 3 --warmup 1 --cpu-baseline 0 --rows-scale 0 --sssp-roots 2 \
    > gpurun_out/r04c/bench_part.json 2> gpurun_out/r04c/bench_part.err
rc=$?; tail -3 gpurun_out/r04c/bench_part.err; cat gpurun_out/r04c/bench_part.json | head -c 3000; exit $rc
