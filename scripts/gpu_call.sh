#!/bin/bash
# Round-4 call d: counter names on gfx950; PageRank time attributable to the top sources of
# the hot pass (TGO_PR_SKIP_BELOW diagnostic: those gathers skipped).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04d
timeout -k 10 120 rocprofv3 -L > gpurun_out/r04d/counters.txt 2>&1; echo "rocprofv3 -L exit $?"
bash scripts/gpu_pr_ab.sh r04d_skip "TGO_PR_SKIP_BELOW=0" "TGO_PR_SKIP_BELOW=1024" "TGO_PR_SKIP_BELOW=4096" \
    "TGO_PR_SKIP_BELOW=16384" "TGO_PR_SKIP_BELOW=65536" "TGO_PR_SKIP_BELOW=131072" "TGO_PR_SKIP_BELOW=393216" \
    > gpurun_out/r04d/skip.log 2>&1
rc=$?; cat gpurun_out/r04d/skip.log; exit $rc
