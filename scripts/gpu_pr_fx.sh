#!/bin/bash
# Fixed-point hot pass A/B on RMAT-24 (pr_probe.py): the slot form (TGO_PR_FX=0) first, then
# super-tile sizes; ms/update, reproducibility and L1 against the slot form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-prfx}
OUT=gpurun_out/$TAG; mkdir -p $OUT
PR_PROBE_VARIANTS=${PR_PROBE_VARIANTS:-'[{"TGO_PR_FX": "0"}, {"TGO_PR_FX": "1"}, {"TGO_PR_FX": "1", "TGO_PR_FX_E": "32768"}, {"TGO_PR_FX": "1", "TGO_PR_FX_E": "131072"}, {"TGO_PR_FX": "1", "TGO_PR_FX_E": "262144"}, {"TGO_PR_FX": "0"}]'} \
  timeout -k 10 400 python3 -u scripts/pr_probe.py 24 20 > $OUT/probe.log 2>&1
rc=$?; cat $OUT/probe.log; exit $rc
