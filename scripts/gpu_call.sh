#!/bin/bash
# Round-3 call m: rows load with device-resident decoded entries (tests + probe); SSSP delta sweep
# under the device loop.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03m; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_assembly.py tests/test_gpu_decode.py tests/test_gpu_scan.py > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 300 python3 scripts/rows_probe.py 20 > $OUT/rows.log 2>&1
rc=$?; grep -E "finish|load [0-9]" $OUT/rows.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/sssp_probe.py 24 12,16,24,31,48,64 > $OUT/sssp_delta.log 2>&1
rc=$?; grep -E "^delta" $OUT/sssp_delta.log; exit $rc
