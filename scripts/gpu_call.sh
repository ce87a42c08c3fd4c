#!/bin/bash
# Single-source BFS with the 256-entry serial scan: BFS parity (one-GPU, full size, scale 27,
# partitioned), the smoke test and the bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04zc
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_scale27.py tests/test_gpu_distributed.py tests/test_gpu_scan.py \
    tests/test_gpu_decode.py -k "bfs or shortest or load_rows or scan" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -2 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$T/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; cut -c1-300 gpurun_out/$T/bench.json; exit $rc
