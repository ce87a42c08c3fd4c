#!/bin/bash
# SSSP pull form of finished buckets' heavy entries: parity, then an A/B of the push and pull
# forms at RMAT-24 (sssp_once.py, 4 roots) with the kernel split of the pull run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04p
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "sssp or delta" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
SSSP_BINS=1 SSSP_PULL=0,0.002,0.01,0.05 timeout -k 10 300 python -u scripts/sssp_once.py 24 4 > gpurun_out/$T/ab.log 2>&1
rc=$?; cat gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
TGO_DS_PULL=0.01 timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py \
    -k "config5" > gpurun_out/$T/full5.log 2>&1
rc=$?; tail -3 gpurun_out/$T/full5.log; exit $rc
