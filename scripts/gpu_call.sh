#!/bin/bash
# Multi-source pull: the wave-cooperative list threshold (TGO_MS_COOP) A/B on the sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04z7
mkdir -p gpurun_out/$T
for v in 64 16 32 128 256 64 16 32 128 256; do
    TGO_MS_COOP=$v timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; echo "coop $v: $(tail -1 gpurun_out/$T/ab.tmp)" | cut -c1-110 | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
