#!/bin/bash
# Light push (no reached-mask read while few vertices are reached; optionally no candidate
# probe), 4-in-flight per-source entries: parity, A/B of the sweep, kernel timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04s
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_distributed.py tests/test_gpu_fullsize.py -k "multi or msbfs or config3" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for v in "TGO_MS_PUSH_LIGHT=0" "TGO_MS_PUSH_LIGHT=0.0625" "TGO_MS_PUSH_PROBE=0" "TGO_MS_PUSH_LIGHT=0" "TGO_MS_PUSH_LIGHT=0.0625" "TGO_MS_PUSH_PROBE=0"; do
    env $v timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; echo "$v: $(tail -1 gpurun_out/$T/ab.tmp)" | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
TGO_MS_PUSH_PROBE=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/kt -o ms -- \
    python3 scripts/ms_probe.py 24 3 > gpurun_out/$T/probe.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 scripts/ktimeline.py gpurun_out/$T/kt ms_seed > gpurun_out/$T/timeline.txt
rc=$?; rm -rf gpurun_out/$T/kt; head -30 gpurun_out/$T/timeline.txt; exit $rc
