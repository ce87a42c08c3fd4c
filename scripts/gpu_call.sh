#!/bin/bash
# Round-3 call aa: one-pass exact per-source entries for the source split (parity at the
# default and a forced 30 % budget, probe, partitioned bench).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03aa; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py -k "multi_source" tests/test_gpu_fullsize.py::test_config3_rmat24_msbfs_sweep tests/test_gpu_distributed.py > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TGO_MS_SPLIT=0.3 timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_distributed.py -k "msbfs or multi_source" > $OUT/gpu_tests_split.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests_split.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/ms_probe.py 24 5 > $OUT/ms.log 2>&1; rc=$?; grep msbfs $OUT/ms.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 200 python3 scripts/ms_probe.py 24 1 > $OUT/ms_trace.log 2>&1; grep split $OUT/ms_trace.log | head -2
timeout -k 10 400 python3 bench.py --partitioned --cpu-baseline 0 --sssp-roots 0 --rows-scale 0 > $OUT/bench_part.json 2> $OUT/bench_part.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bench_part.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_part.json')); print('native partitioned', d['value'], d['ms_per_step'])"
