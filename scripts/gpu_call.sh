#!/bin/bash
# Round-4 call n: partitioned drivers read their per-level counts through the mapped counter
# page (tests, per-level probe, partitioned bench line at world 1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04n
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_distributed.py tests/test_gpu_fullsize.py -k "partitioned or native or distributed or sweep or msbfs" \
    > gpurun_out/r04n/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04n/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ms_levels.py 24 5 > gpurun_out/r04n/ms_levels.log 2>&1
rc=$?; grep -E "sweep|level" gpurun_out/r04n/ms_levels.log | grep -v Exception | tail -12; [ $rc -eq 0 ] || exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 600 python3 bench.py --partitioned --steps 3 --warmup 1 --cpu-baseline 0 --rows-scale 0 --sssp-roots 2 \
    > gpurun_out/r04n/bench_part.json 2> gpurun_out/r04n/bench_part.err
rc=$?; tail -2 gpurun_out/r04n/bench_part.err; python3 -c "
import json; d=json.load(open('gpurun_out/r04n/bench_part.json')); print('GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'], 'sssp', d['sssp'])"
exit $rc
