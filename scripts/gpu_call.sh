#!/bin/bash
# Round-3 call q: tgo_load_csr tests; staged push kernels (ms_push, td_expand) with tile appends: parity + probes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03q; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 800 $T tests/test_gpu_load_csr.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/ms_probe.py 24 5 > $OUT/ms.log 2>&1; rc=$?; grep msbfs $OUT/ms.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bfs_probe.py 24 8 > $OUT/bfs.log 2>&1; rc=$?; tail -8 $OUT/bfs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms -o run -- python3 scripts/ms_probe.py 24 3 > $OUT/ms_prof.log 2>&1
rc=$?; rm -f $OUT/ms/run_kernel_trace.csv; exit $rc
