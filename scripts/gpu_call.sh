#!/bin/bash
# Fused push-level prep (sweep A/B), and one delta-SSSP run kernel by kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04v
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "multi" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -2 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; tail -1 gpurun_out/$T/ab.tmp | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/kt -o ss -- \
    python3 scripts/sssp_once.py 24 1 > gpurun_out/$T/sssp.log 2>&1
rc=$?; tail -2 gpurun_out/$T/sssp.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/ktimeline.py gpurun_out/$T/kt ds_loop_seed > gpurun_out/$T/sssp_timeline.txt
rc=$?; rm -rf gpurun_out/$T/kt; tail -14 gpurun_out/$T/sssp_timeline.txt; exit $rc
