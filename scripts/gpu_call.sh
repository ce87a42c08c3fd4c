#!/bin/bash
# Round-4 call e: request-rate counters of the PageRank kernels and the gather ceiling probe.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_pmc_pr.sh r04e_pmc > gpurun_out/r04e_pmc.log 2>&1
rc=$?; tail -20 gpurun_out/r04e_pmc.log; exit $rc
