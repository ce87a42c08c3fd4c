#!/bin/bash
# Multi-source pull: long-list trip size / first-trip ramp / short-list step A/B on the sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04z4
mkdir -p gpurun_out/$T
for v in "TGO_MS_LONG=4" "TGO_MS_LONG=1" "TGO_MS_LONG=2" "TGO_MS_LONG=8" "TGO_MS_RAMP=1" "TGO_MS_STEP=4" "TGO_MS_STEP=16" \
         "TGO_MS_LONG=4" "TGO_MS_LONG=1" "TGO_MS_LONG=2" "TGO_MS_LONG=8" "TGO_MS_RAMP=1" "TGO_MS_STEP=4" "TGO_MS_STEP=16"; do
    env $v timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; echo "$v: $(tail -1 gpurun_out/$T/ab.tmp)" | cut -c1-120 | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
