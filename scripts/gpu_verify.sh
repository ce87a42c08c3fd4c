#!/bin/bash
# Verification of the committed tree: full GPU suite, smoke(), default bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-verify}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/$T/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; echo "bench exit $rc"; python3 -c "import json; d=json.load(open('gpurun_out/$T/bench.json')); print(d['value'], d['pagerank_s_per_iter'], d['roofline']['frac'], d['single_source_gteps_hmean'])"; exit $rc
