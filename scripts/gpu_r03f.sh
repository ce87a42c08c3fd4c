#!/bin/bash
# Round-3 call f: full GPU suite (native partitioned driver, extraction unroll, level_prep
# grid-stride), sweep / SSSP probes, the RMAT-27 one-GPU check, the partitioned bench at N=1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ms_probe.py 24 3 > $OUT/ms_probe.log 2>&1; tail -1 $OUT/ms_probe.log
TGO_TRACE=1 TGO_MS_DIAG=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 1 > $OUT/ms_diag.log 2>&1; grep -E "upload|assembly|pull" $OUT/ms_diag.log | head -30
TGO_TRACE=1 PR_PROBE_DEFAULT_ONLY=1 timeout -k 10 300 python3 scripts/pr_probe.py 24 20 > $OUT/pr_load.log 2>&1; grep -E "upload|assembly|ms_per" $OUT/pr_load.log | head
timeout -k 10 300 python3 scripts/sssp_probe.py 24 0 > $OUT/sssp_probe.log 2>&1; tail -2 $OUT/sssp_probe.log
timeout -k 10 400 python3 bench.py --partitioned --cpu-baseline 0 --sssp-roots 0 --rows-scale 0 > $OUT/bench_part.json 2> $OUT/bench_part.err
echo "partitioned bench rc $?"; python3 -c "import json; d=json.load(open('$OUT/bench_part.json')); print(d['value'], d['pagerank_s_per_iter'], d['config'].get('msbfs_driver'), d['partition'])"
timeout -k 10 480 python3 -u scripts/scale27_check.py 27 64 > $OUT/scale27.json 2> $OUT/scale27.err; echo s27 rc $?; cat $OUT/scale27.json
