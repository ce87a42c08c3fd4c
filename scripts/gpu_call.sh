#!/bin/bash
# Round-3 call h: device-resident assembly handoff (assembly tests + load trace), MS-BFS
# cold-only frontier filter (parity under the filter, TGO_MS_FILTER_FROM A/B), partitioned
# bench at N=1 native vs Python driver after the pinned-count fix.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03h; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_assembly.py tests/test_gpu_parity.py > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TGO_MS_FILTER_FROM=1000 timeout -k 10 300 $T tests/test_gpu_parity.py -k "multi_source" tests/test_gpu_fullsize.py::test_config3_rmat24_msbfs_sweep > $OUT/gpu_filter_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_filter_tests.log; [ $rc -eq 0 ] || exit $rc
for H in -1 0 131072 262144 393216 1048576; do
  TGO_MS_FILTER_FROM=$H timeout -k 10 200 python3 scripts/ms_probe.py 24 5 >> $OUT/ms_filter.log 2>&1 || exit 1
done
grep msbfs $OUT/ms_filter.log
TGO_TRACE=1 PR_PROBE_DEFAULT_ONLY=1 timeout -k 10 300 python3 scripts/pr_probe.py 24 20 > $OUT/pr_load.log 2>&1; grep -E "upload|assembl|cold|ms_per" $OUT/pr_load.log | head -20
timeout -k 10 400 python3 bench.py --partitioned --cpu-baseline 0 --sssp-roots 0 --rows-scale 0 > $OUT/bench_part.json 2> $OUT/bench_part.err
rc=$?; echo "partitioned bench rc $rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_part.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_part.json')); print('native', d['value'], d['ms_per_step'])"
timeout -k 10 400 python3 bench.py --partitioned --native 0 --cpu-baseline 0 --sssp-roots 0 --rows-scale 0 > $OUT/bench_part_py.json 2> $OUT/bench_part_py.err
python3 -c "import json; d=json.load(open('$OUT/bench_part_py.json')); print('python driver', d['value'], d['ms_per_step'])"
