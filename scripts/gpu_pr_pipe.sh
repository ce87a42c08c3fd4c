#!/bin/bash
# A/B of the persistent pipelined PageRank gathers (TGO_PR_PIPE) on RMAT-24: ms/update and
# bitwise equality of the ranks across the two kernels; then the PageRank parity tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prpipe
for p in 0 1; do
  TGO_PR_PIPE=$p PR_PROBE_DEFAULT_ONLY=1 PR_PROBE_SAVE=gpurun_out/prpipe/pr$p.sha timeout -k 10 300 \
      python3 scripts/pr_probe.py 24 20 > gpurun_out/prpipe/probe$p.log 2>&1 || { tail -5 gpurun_out/prpipe/probe$p.log; exit 1; }
  echo "pipe=$p"; tail -1 gpurun_out/prpipe/probe$p.log
done
cmp -s gpurun_out/prpipe/pr0.sha gpurun_out/prpipe/pr1.sha && echo "bitwise equal True" || echo "bitwise equal False"
if [ -n "$PIPE_TESTS" ]; then
  TGO_PR_PIPE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "pagerank" --timeout 300 --timeout-method thread > gpurun_out/prpipe/tests.log 2>&1
  rc=$?; tail -2 gpurun_out/prpipe/tests.log; exit $rc
fi
