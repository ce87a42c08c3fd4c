#!/bin/bash
# Round-3 call s2: source split, transposed per-source counts (parity + budget A/B).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03s4; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py -k "multi_source" tests/test_gpu_fullsize.py::test_config3_rmat24_msbfs_sweep > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 0.005; do TGO_MS_SPLIT=$f timeout -k 10 200 python3 scripts/ms_probe.py 24 5 > $OUT/ms_split_$f.log 2>&1 || exit 1; grep msbfs $OUT/ms_split_$f.log; done
TGO_TRACE=1 TGO_MS_DIAG=1 timeout -k 10 200 python3 scripts/ms_probe.py 24 1 > $OUT/ms_diag.log 2>&1 || exit 1
grep -E "split|pull:" $OUT/ms_diag.log | head -6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms -o run -- python3 scripts/ms_probe.py 24 3 > $OUT/ms_prof.log 2>&1
rc=$?; rm -f $OUT/ms/run_kernel_trace.csv; exit $rc
