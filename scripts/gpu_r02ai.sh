#!/bin/bash
# Device-staged decode with device compaction; PageRank prefetch / LDS-pad A/B; bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02ai
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_scan.py tests/test_gpu_fullsize.py \
    tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02ai/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02ai/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pr_ab.sh prab_ai "TGO_PR_LDSPAD=0" "TGO_PR_LDSPAD=1" "TGO_PR_PF=0 TGO_PR_LDSPAD=0" "TGO_PR_LDSPAD=0 TGO_PR_FOLD=1" || exit 1
TGO_PR_LDSPAD=0 timeout -k 10 500 python3 bench.py > gpurun_out/r02ai/bench.json 2> gpurun_out/r02ai/bench.err
rc=$?; echo "bench exit $rc"; tail -2 gpurun_out/r02ai/bench.err; exit $rc
