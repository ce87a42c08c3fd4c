#!/bin/bash
# Round-4 call f2: the LDS window pass (wave items, prefetch): parity tests, then A/B of window sizes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "pagerank" tests/test_gpu_trace.py > gpurun_out/r04f/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04f/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_assembly.py -k "pagerank" "tests/test_gpu_fullsize.py::test_config3_rmat24_pagerank_capped" \
    > gpurun_out/r04f/gpu_tests2.log 2>&1
rc=$?; tail -5 gpurun_out/r04f/gpu_tests2.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pr_ab.sh r04f_win "TGO_PR_WIN=0" "TGO_PR_WIN=12032" "TGO_PR_WIN=8192" "TGO_PR_WIN=4096" "TGO_PR_WIN=12032 TGO_PR_SKIP_BELOW=393216" \
    > gpurun_out/r04f/ab.log 2>&1
rc=$?; cat gpurun_out/r04f/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py -k "native or pagerank" > gpurun_out/r04f/gpu_tests3.log 2>&1
rc=$?; tail -5 gpurun_out/r04f/gpu_tests3.log; [ $rc -eq 0 ] || exit $rc
TGO_TRACE=1 timeout -k 10 300 python3 scripts/load27_trace.py 27 gpurun_out/r04f/load27_trace.json > gpurun_out/r04f/load27.log 2>&1
rc=$?; grep -v "level" gpurun_out/r04f/load27.log | tail -40; exit $rc
