#!/bin/bash
# Round-4 call h: binned delta-stepping (piles + done filter) parity, A/B against the bitmap
# loop with a kernel trace; scale-27 load with allocation timings.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "sssp or delta" tests/test_gpu_fullsize.py::test_config5_rmat24_weighted_sssp \
    > gpurun_out/r04h/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04h/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
SSSP_BINS=1,0 TGO_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04h/sssp_kt -o run -- \
    python3 scripts/sssp_once.py 24 2 > gpurun_out/r04h/sssp_once.log 2>&1
rc=$?; grep -E "root|delta" gpurun_out/r04h/sssp_once.log | tail -12; [ $rc -eq 0 ] || exit $rc
python3 scripts/ktrace.py gpurun_out/r04h/sssp_kt ds_relax_dev,ds_extract 12 > gpurun_out/r04h/sssp_ktrace.txt; grep -E "ds_|dispatches" gpurun_out/r04h/sssp_ktrace.txt
TGO_TRACE=1 timeout -k 10 300 python3 scripts/load27_trace.py 27 gpurun_out/r04h/load27_trace.json > gpurun_out/r04h/load27.log 2>&1
rc=$?; grep -v "level" gpurun_out/r04h/load27.log | grep -E "load27|tmp|cut|rekey|assembly|cold build|upload" | tail -45; exit $rc
