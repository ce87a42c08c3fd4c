#!/bin/bash
# Round-3 call o: unrolled / mask-skipping extraction (every frontier kernel): parity tests and probes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03o; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/ms_probe.py 24 5 > $OUT/ms.log 2>&1; rc=$?; grep msbfs $OUT/ms.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/sssp_probe.py 24 0 > $OUT/sssp.log 2>&1; rc=$?; grep "^delta" $OUT/sssp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bfs_probe.py > $OUT/bfs.log 2>&1; rc=$?; tail -3 $OUT/bfs.log; exit $rc
