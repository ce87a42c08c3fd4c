#!/bin/bash
# Partitioned sweep: settle-summed per-source entries and fused settle prep — the distributed
# parity tests, then the world-1 partitioned bench against the one-GPU sweep probe.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04y
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
    tests/test_gpu_fullsize.py -k "msbfs or multi or partitioned or config3" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --partitioned --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 \
    > gpurun_out/$T/bench_part.json 2> gpurun_out/$T/bench_part.err
rc=$?; cut -c1-600 gpurun_out/$T/bench_part.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/$T/bench_part.err; exit $rc; }
timeout -k 10 300 python3 scripts/ms_levels.py 24 3 > gpurun_out/$T/ms_levels.log 2>&1
rc=$?; head -14 gpurun_out/$T/ms_levels.log; exit $rc
