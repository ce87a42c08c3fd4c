#!/bin/bash
# One development GPU call: selected GPU tests, then PageRank hot-tile A/B on RMAT-24.
# usage: bash scripts/gpu_r03_step.sh <tag> "<pytest args>" [A/B variants...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS \
      > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -15 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
[ $# -gt 0 ] && bash scripts/gpu_pr_ab.sh $TAG/ab "$@"
exit 0
