#!/bin/bash
# Settle-summed per-source entries + target-ranged push: parity (+ the dev cross-check and
# ranged = queue-order), A/B of the range size, the default sweep's kernel timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04t
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_distributed.py -k "multi or msbfs" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
TGO_MS_SRCENT_CHECK=1 TGO_TRACE=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 3 > gpurun_out/$T/check.log 2>&1
rc=$?; grep -c "checked" gpurun_out/$T/check.log; tail -1 gpurun_out/$T/check.log; [ $rc -eq 0 ] || exit $rc
for v in 0 18 16 20 0 18 16 20; do
    TGO_MS_PUSH_RANGE=$v timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; echo "range $v: $(tail -1 gpurun_out/$T/ab.tmp)" | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/kt -o ms -- \
    python3 scripts/ms_probe.py 24 3 > gpurun_out/$T/probe.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 scripts/ktimeline.py gpurun_out/$T/kt ms_seed > gpurun_out/$T/timeline.txt
rc=$?; rm -rf gpurun_out/$T/kt; head -36 gpurun_out/$T/timeline.txt; exit $rc
