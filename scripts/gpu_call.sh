#!/bin/bash
# Delta SSSP: device-loop batch size A/B (steps enqueued per host read of the loop state).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04w
mkdir -p gpurun_out/$T
for b in 8 16 32 64 8 16 32 64; do
    TGO_DS_BATCH=$b timeout -k 10 300 python3 scripts/sssp_once.py 24 4 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/$T/ab.tmp; exit $rc; }
    grep "GTEPS" gpurun_out/$T/ab.tmp | sed "s/^/batch $b: /" | tee -a gpurun_out/$T/ab.log
done
