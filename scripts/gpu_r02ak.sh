#!/bin/bash
# Non-temporal per-row streams in the PageRank gathers; hot-head size re-sweep; PR parity tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02ak
bash scripts/gpu_pr_ab.sh prab_ak "TGO_PR_NT=1" "TGO_PR_NT=0" "TGO_PR_NT=1 TGO_PR_HOT=393216" "TGO_PR_NT=1 TGO_PR_HOT=262144" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "pagerank or PageRank or pr_" \
    --timeout 200 --timeout-method thread > gpurun_out/r02ak/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r02ak/gpu_tests.log; exit $rc
