#!/bin/bash
# Settle sums only ahead of a possible pull level, ranged push off: parity of the sweep paths,
# the sweep A/B, and the bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04u
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_distributed.py tests/test_gpu_fullsize.py -k "multi or msbfs or config3" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; tail -1 gpurun_out/$T/ab.tmp | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; cat gpurun_out/$T/bench.json; exit $rc
