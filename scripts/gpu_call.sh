#!/bin/bash
# Sweep: no seed-degree readback, queue-less settle ahead of a pull level — parity, the sweep
# time, its kernel timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04z3
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_distributed.py tests/test_gpu_fullsize.py -k "multi or msbfs or config3" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
    timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; tail -1 gpurun_out/$T/ab.tmp | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/kt -o ms -- \
    python3 scripts/ms_probe.py 24 3 > gpurun_out/$T/probe.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 scripts/ktimeline.py gpurun_out/$T/kt ms_seed > gpurun_out/$T/timeline.txt
rc=$?; rm -rf gpurun_out/$T/kt; tail -22 gpurun_out/$T/timeline.txt; exit $rc
