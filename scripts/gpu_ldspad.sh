#!/bin/bash
# A/B of the padded LDS tile (TGO_PR_LDSPAD) in the cache-blocked PageRank gathers on RMAT-24:
# ms/update, bitwise equality of the ranks, and per-kernel times of the padded run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ldspad
for p in 0 1; do
  TGO_PR_LDSPAD=$p PR_PROBE_DEFAULT_ONLY=1 PR_PROBE_SAVE=gpurun_out/ldspad/pr$p.sha timeout -k 10 300 \
      python3 scripts/pr_probe.py 24 20 > gpurun_out/ldspad/probe$p.log 2>&1 || { tail -5 gpurun_out/ldspad/probe$p.log; exit 1; }
  echo "pad=$p"; tail -1 gpurun_out/ldspad/probe$p.log
done
cmp -s gpurun_out/ldspad/pr0.sha gpurun_out/ldspad/pr1.sha && echo "bitwise equal True" || echo "bitwise equal False"
TGO_PR_LDSPAD=1 PR_PROBE_DEFAULT_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/ldspad -o prof -- python3 scripts/pr_probe.py 24 20 > gpurun_out/ldspad/prof.log 2>&1
rc=$?; rm -f gpurun_out/ldspad/prof_kernel_trace.csv; echo "prof exit $rc"; exit $rc
