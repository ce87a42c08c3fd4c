#!/bin/bash
# Multi-source sweep kernel by kernel: the probe's last sweep under --kernel-trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04q
mkdir -p gpurun_out/$T
TGO_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/kt -o ms -- \
    python3 scripts/ms_probe.py 24 3 > gpurun_out/$T/probe.log 2>&1
rc=$?; tail -5 gpurun_out/$T/probe.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/ktimeline.py gpurun_out/$T/kt ms_seed > gpurun_out/$T/timeline.txt
rc=$?; rm -rf gpurun_out/$T/kt; cat gpurun_out/$T/timeline.txt; exit $rc
