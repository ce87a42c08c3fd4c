#!/bin/bash
# Partitioned push straight into the next masks for owned targets: distributed parity (world
# 1/2/4 in-process, scale 27 world 2) and the world-1 partitioned bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04z8
mkdir -p gpurun_out/$T
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
    tests/test_gpu_fullsize.py tests/test_gpu_scale27.py -k "msbfs or multi or partitioned or world" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --partitioned --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 \
    > gpurun_out/$T/bench_part.json 2> gpurun_out/$T/bench_part.err
rc=$?; cut -c1-300 gpurun_out/$T/bench_part.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ms_levels.py 24 3 > gpurun_out/$T/ms_levels.log 2>&1
rc=$?; head -14 gpurun_out/$T/ms_levels.log; exit $rc
