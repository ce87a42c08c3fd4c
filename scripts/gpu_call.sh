#!/bin/bash
# Round-4 final code (256-entry bottom-up serial scan): the full GPU suite, smoke(), the bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04fin2
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$T/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; cut -c1-300 gpurun_out/$T/bench.json; exit $rc
