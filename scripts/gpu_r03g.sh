#!/bin/bash
# Round-3 call g: device row assembly tests + configs[1] full-size rows test, MS-BFS long-list
# diagnostics, partitioned bench at N=1 (native driver), rows load trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_assembly.py \
    tests/test_gpu_decode.py tests/test_gpu_scan.py tests/test_gpu_fullsize.py \
    > $OUT/gpu_tests.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 TGO_MS_DIAG=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 1 > $OUT/ms_diag.log 2>&1; grep -E "pull" $OUT/ms_diag.log | head -8
TGO_TRACE=1 PR_PROBE_DEFAULT_ONLY=1 timeout -k 10 300 python3 scripts/pr_probe.py 24 20 > $OUT/pr_load.log 2>&1; grep -E "upload|assembly|cold|ms_per" $OUT/pr_load.log | head -12
timeout -k 10 400 python3 bench.py --partitioned --cpu-baseline 0 --sssp-roots 0 --rows-scale 0 > $OUT/bench_part.json 2> $OUT/bench_part.err
rc=$?; echo "partitioned bench rc $rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_part.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_part.json')); print(d['value'], d['pagerank_s_per_iter'], d['config'].get('msbfs_driver'), d['partition'])"
timeout -k 10 400 python3 bench.py --partitioned --native 0 --cpu-baseline 0 --sssp-roots 0 --rows-scale 0 > $OUT/bench_part_py.json 2> $OUT/bench_part_py.err
python3 -c "import json; d=json.load(open('$OUT/bench_part_py.json')); print('python driver', d['value'], d['pagerank_s_per_iter'])"
