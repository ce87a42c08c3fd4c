#!/bin/bash
# Round-3 call k: device-driven delta-stepping loop (parity + probe, A/B against the host
# loop), partitioned MS-BFS over active rows (tests + bench native vs one-GPU).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03k; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_fullsize.py::test_config5_rmat24_weighted_sssp tests/test_gpu_distributed.py > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 300 python3 scripts/sssp_probe.py 24 0 > $OUT/sssp_dev.log 2>&1
rc=$?; grep -E "^delta|device loop" $OUT/sssp_dev.log | tail -2; [ $rc -eq 0 ] || exit $rc
TGO_DS_HOSTLOOP=1 timeout -k 10 300 python3 scripts/sssp_probe.py 24 0 > $OUT/sssp_host.log 2>&1
rc=$?; grep -E "^delta" $OUT/sssp_host.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ss -o run -- python3 scripts/sssp_probe.py 24 0 > $OUT/ss_prof.log 2>&1
rc=$?; tail -1 $OUT/ss_prof.log; rm -f $OUT/ss/run_kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --partitioned --cpu-baseline 0 --sssp-roots 0 --rows-scale 0 > $OUT/bench_part.json 2> $OUT/bench_part.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bench_part.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_part.json')); print('native partitioned', d['value'], d['ms_per_step'])"
timeout -k 10 200 python3 scripts/ms_probe.py 24 5 > $OUT/ms.log 2>&1; grep msbfs $OUT/ms.log
