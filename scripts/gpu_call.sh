#!/bin/bash
# Pull-shape sweeps equal (new test), then split budget / direction switch A/B with the
# 64-entry long-list trips.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04z9
mkdir -p gpurun_out/$T
timeout -k 10 800 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
    -k "pull_shapes or settle_sums" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for v in "TGO_MS_SPLIT=0.005" "TGO_MS_SPLIT=0" "TGO_MS_SPLIT=0.002" "TGO_MS_SPLIT=0.01" "TGO_MS_SPLIT=0.02" \
         "TGO_MS_ALPHA=8" "TGO_MS_ALPHA=16" "TGO_MS_ALPHA=24" \
         "TGO_MS_SPLIT=0.005" "TGO_MS_SPLIT=0" "TGO_MS_SPLIT=0.002" "TGO_MS_SPLIT=0.01" "TGO_MS_SPLIT=0.02" \
         "TGO_MS_ALPHA=8" "TGO_MS_ALPHA=16" "TGO_MS_ALPHA=24"; do
    env $v timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; echo "$v: $(tail -1 gpurun_out/$T/ab.tmp)" | cut -c1-110 | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
