#!/bin/bash
# Round-4 call m: split first pull level (hot walk + blocked cold pass) parity and A/B; the
# own-slice bypass per-level probe and partitioned bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04m
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "multi_source or msbfs" tests/test_gpu_fullsize.py -k "msbfs or multi" \
    > gpurun_out/r04m/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04m/tests.log; [ $rc -eq 0 ] || exit $rc
for V in 0 1; do
  TGO_MS_COLD=$V TGO_TRACE=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/r04m/ms_cold$V.log 2>&1
  rc=$?; echo "== TGO_MS_COLD=$V"; grep -E "msbfs scale|cold_layout" gpurun_out/r04m/ms_cold$V.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 scripts/ms_levels.py 24 5 > gpurun_out/r04m/ms_levels.log 2>&1
rc=$?; grep -E "sweep|level" gpurun_out/r04m/ms_levels.log | grep -v Exception | tail -12; [ $rc -eq 0 ] || exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 600 python3 bench.py --partitioned --steps 3 --warmup 1 --cpu-baseline 0 --rows-scale 0 --sssp-roots 2 \
    > gpurun_out/r04m/bench_part.json 2> gpurun_out/r04m/bench_part.err
rc=$?; tail -2 gpurun_out/r04m/bench_part.err; python3 -c "
import json; d=json.load(open('gpurun_out/r04m/bench_part.json')); print('GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'], 'sssp', d['sssp'])"
exit $rc
