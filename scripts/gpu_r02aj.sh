#!/bin/bash
# PageRank block descriptors: parity tests, A/B against the non-prefetching kernels, profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02aj
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py \
    -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02aj/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02aj/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pr_ab.sh prab_aj "TGO_PR_PF=1" "TGO_PR_PF=0" || exit 1
PR_PROBE_DEFAULT_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r02aj -o prof -- python3 scripts/pr_probe.py 24 20 > gpurun_out/r02aj/prof.log 2>&1
rc=$?; rm -f gpurun_out/r02aj/prof_kernel_trace.csv; echo "prof exit $rc"; exit $rc
