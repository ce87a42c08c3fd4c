#!/bin/bash
# Round-4 call j: load path changes (pinned-bounce downloads, huge-page host vectors, threaded
# id fill, moved host vectors) against the assembly / full-size tests and the scale-27 trace;
# delta SSSP parity with the tuning keys.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04j
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1 | head -2
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "sssp or delta" tests/test_gpu_assembly.py tests/test_gpu_fullsize.py \
    > gpurun_out/r04j/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04j/tests.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 300 python3 scripts/load27_trace.py 27 gpurun_out/r04j/load27_trace.json > gpurun_out/r04j/load27.log 2>&1
rc=$?; grep -v "level" gpurun_out/r04j/load27.log | tail -60; exit $rc
