#!/bin/bash
# Device-decode parity, pipelined-PageRank A/B, partitioned-path profile (one call).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02af
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_scan.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02af/decode_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02af/decode_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pr_pipe.sh && bash scripts/gpu_part_prof.sh
