#!/bin/bash
# Staged multi-source push, bit-sliced per-source entries, one-lane-per-seed seeding: parity,
# then the sweep kernel by kernel and the probe's sweep time.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04r
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_distributed.py tests/test_gpu_fullsize.py -k "multi or msbfs or config3" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/kt -o ms -- \
    python3 scripts/ms_probe.py 24 3 > gpurun_out/$T/probe.log 2>&1
rc=$?; tail -5 gpurun_out/$T/probe.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/ktimeline.py gpurun_out/$T/kt ms_seed > gpurun_out/$T/timeline.txt
rc=$?; rm -rf gpurun_out/$T/kt; cat gpurun_out/$T/timeline.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/probe_plain.log 2>&1
rc=$?; tail -2 gpurun_out/$T/probe_plain.log; exit $rc
