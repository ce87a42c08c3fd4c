#!/bin/bash
# Round-4 call k: PageRank layout fetch path (tests + scale-27 trace); per-level sweep, one-GPU
# against partitioned world 1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04k
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "pagerank" tests/test_gpu_assembly.py tests/test_gpu_fullsize.py -k "pagerank or layout or cold or assembly" \
    > gpurun_out/r04k/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04k/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ms_levels.py 24 5 > gpurun_out/r04k/ms_levels.log 2>&1
rc=$?; tail -16 gpurun_out/r04k/ms_levels.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 300 python3 scripts/load27_trace.py 27 gpurun_out/r04k/load27_trace.json > gpurun_out/r04k/load27.log 2>&1
rc=$?; grep -v "level" gpurun_out/r04k/load27.log | grep -E "load27|cold|upload|assembly" | tail -20; exit $rc
