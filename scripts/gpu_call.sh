#!/bin/bash
# Round-3 call ab: PageRank layout knobs A/B with the round-3 code.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_pr_ab.sh r03ab "TGO_PR_HOT=393216" "TGO_PR_HOT=524288 TGO_PR_SEG=393216" \
    "TGO_PR_HOT=393216 TGO_PR_SEG=524288" "TGO_PR_HOT=262144 TGO_PR_SEG=393216" "TGO_PR_HOT_TILE=8192" \
    "TGO_PR_HOT=393216 TGO_PR_SEG=262144" > gpurun_out/r03ab.log 2>&1
rc=$?; cat gpurun_out/r03ab.log; exit $rc
