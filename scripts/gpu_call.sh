#!/bin/bash
# Round-4 call i: binned delta-stepping variants (pile-scan threshold, done filter) A/B with a
# kernel trace, parity first.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04i
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "sssp or delta" tests/test_gpu_fullsize.py::test_config5_rmat24_weighted_sssp \
    > gpurun_out/r04i/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04i/tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for V in "TGO_DS_BINS=0" "TGO_DS_BINS=1" "TGO_DS_DONE=0" "TGO_DS_PILE_SCAN=0.25" "TGO_DS_PILE_SCAN=0.01" "TGO_DS_PILE_SCAN=0.01 TGO_DS_DONE=0"; do
  env $V SSSP_BINS=-1 TGO_TRACE=1 timeout -k 10 300 python3 scripts/sssp_once.py 24 3 > gpurun_out/r04i/v$i.log 2>&1
  rc=$?; echo "== $V"; grep -E "root" gpurun_out/r04i/v$i.log; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
TGO_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04i/sssp_kt -o run -- \
    python3 scripts/sssp_once.py 24 2 > gpurun_out/r04i/sssp_once.log 2>&1
rc=$?; grep -E "delta" gpurun_out/r04i/sssp_once.log | tail -4; exit $rc
