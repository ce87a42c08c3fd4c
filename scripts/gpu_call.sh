#!/bin/bash
# Round-3 call z: smoke(), SSSP (heavy entries skip the source's distance reload): parity +
# probe, and the partitioned world-1 sweep timeline (kernel trace).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03z; mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py -k "sssp" tests/test_gpu_fullsize.py::test_config5_rmat24_weighted_sssp tests/test_gpu_load_csr.py > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/sssp_probe.py 24 0 > $OUT/sssp.log 2>&1; rc=$?; grep "^delta" $OUT/sssp.log; [ $rc -eq 0 ] || exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/pp -o run -- \
    python3 bench.py --partitioned --steps 2 --warmup 1 --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 \
    > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -2 $OUT/bench.err; exit $rc
