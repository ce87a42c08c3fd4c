#!/bin/bash
# GPU check used during development: parity tests, then a profiled bench run.
# usage (on the GPU box): bash scripts/gpu_check.sh <tag> [bench args...]
TAG=${1:-dev}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/gpu_tests.log
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- \
    python3 bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; echo "bench exit $rc"; tail -4 gpurun_out/$TAG/bench.err; cat gpurun_out/$TAG/bench.json
exit $rc
