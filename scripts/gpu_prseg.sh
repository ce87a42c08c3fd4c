#!/bin/bash
# Hot-head / segment sizes with the round-2 PageRank kernels, and the no-gather floor.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prseg
PR_PROBE_VARIANTS="$PR_VARIANTS" \
  timeout -k 10 500 python3 scripts/pr_probe.py 24 20 > gpurun_out/prseg/probe.log 2>&1
rc=$?; cat gpurun_out/prseg/probe.log | grep -v "^\[" | tail -16; exit $rc
