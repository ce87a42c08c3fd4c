#!/bin/bash
# GPU parity tests (development runs): bash scripts/gpu_tests.sh <tag> [pytest args...]
TAG=${1:-dev}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; tail -25 gpurun_out/$TAG/gpu_tests.log
exit $rc
