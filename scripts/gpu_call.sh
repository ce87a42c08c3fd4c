#!/bin/bash
# Round-4 call g: full GPU suite (logged), scale-27 load trace with the temporaries cache, the
# one-GPU bench line and the partitioned world-1 bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04g
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    > gpurun_out/r04g/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04g/gpu_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 300 python3 scripts/load27_trace.py 27 gpurun_out/r04g/load27_trace.json > gpurun_out/r04g/load27.log 2>&1
rc=$?; grep -v "level" gpurun_out/r04g/load27.log | tail -45; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r04g/bench.json 2> gpurun_out/r04g/bench.err
rc=$?; tail -2 gpurun_out/r04g/bench.err; head -c 1500 gpurun_out/r04g/bench.json; echo; [ $rc -eq 0 ] || exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 600 python3 bench.py --partitioned --steps 3 --warmup 1 --cpu-baseline 0 --rows-scale 0 --sssp-roots 2 \
    > gpurun_out/r04g/bench_part.json 2> gpurun_out/r04g/bench_part.err
rc=$?; tail -2 gpurun_out/r04g/bench_part.err; python3 -c "
import json; d=json.load(open('gpurun_out/r04g/bench_part.json')); print('GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'], 'sssp', d['sssp'])"
exit $rc
