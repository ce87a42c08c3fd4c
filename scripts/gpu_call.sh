#!/bin/bash
# Multi-source pull with 64-entry long-list trips by default: parity, short-step A/B, the
# bench line and the world-1 partitioned bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04z5
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_distributed.py tests/test_gpu_fullsize.py tests/test_gpu_scale27.py -k "multi or msbfs or config3 or sweep" \
    > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for v in "TGO_MS_STEP=8" "TGO_MS_STEP=4" "TGO_MS_STEP=16" "TGO_MS_STEP=8" "TGO_MS_STEP=4" "TGO_MS_STEP=16"; do
    env $v timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; echo "$v: $(tail -1 gpurun_out/$T/ab.tmp)" | cut -c1-120 | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; cut -c1-400 gpurun_out/$T/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --partitioned --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 \
    > gpurun_out/$T/bench_part.json 2> gpurun_out/$T/bench_part.err
rc=$?; cut -c1-300 gpurun_out/$T/bench_part.json; exit $rc
