#!/bin/bash
# Round-4 call l: own-slice bypass of the partitioned sweep's sparse exchange (tests, per-level
# probe, partitioned bench line at world 1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04l
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_distributed.py > gpurun_out/r04l/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04l/tests.log; [ $rc -eq 0 ] || [ $rc -eq 0 ] || exit $rc
unset RANK WORLD_SIZE LOCAL_RANK MASTER_ADDR MASTER_PORT
TGO_MS_DIAG=1 TGO_TRACE=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 1 > gpurun_out/r04l/ms_diag.log 2>&1
rc=$?; grep -E "ms level|pull:" gpurun_out/r04l/ms_diag.log | tail -12; exit $rc
timeout -k 10 300 python3 scripts/ms_levels.py 24 5 > gpurun_out/r04l/ms_levels.log 2>&1
rc=$?; grep -v Exception gpurun_out/r04l/ms_levels.log | grep -E "sweep|level" | tail -12; [ $rc -eq 0 ] || [ $rc -eq 0 ] || exit $rc
unset RANK WORLD_SIZE LOCAL_RANK MASTER_ADDR MASTER_PORT
TGO_MS_DIAG=1 TGO_TRACE=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 1 > gpurun_out/r04l/ms_diag.log 2>&1
rc=$?; grep -E "ms level|pull:" gpurun_out/r04l/ms_diag.log | tail -12; exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 600 python3 bench.py --partitioned --steps 3 --warmup 1 --cpu-baseline 0 --rows-scale 0 --sssp-roots 2 \
    > gpurun_out/r04l/bench_part.json 2> gpurun_out/r04l/bench_part.err
rc=$?; tail -2 gpurun_out/r04l/bench_part.err; python3 -c "
import json; d=json.load(open('gpurun_out/r04l/bench_part.json')); print('GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'], 'sssp', d['sssp'])"
[ $rc -eq 0 ] || exit $rc
unset RANK WORLD_SIZE LOCAL_RANK MASTER_ADDR MASTER_PORT
TGO_MS_DIAG=1 TGO_TRACE=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 1 > gpurun_out/r04l/ms_diag.log 2>&1
rc=$?; grep -E "ms level|pull:" gpurun_out/r04l/ms_diag.log | tail -12; exit $rc
