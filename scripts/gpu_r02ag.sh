#!/bin/bash
# Full GPU suite (device decode, new host assembly), MS-BFS step A/B, profiled default bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02ag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ag/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02ag/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_msstep.sh || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02ag -o run -- \
    python3 bench.py > gpurun_out/r02ag/bench.json 2> gpurun_out/r02ag/bench.err
rc=$?; echo "bench exit $rc"; tail -3 gpurun_out/r02ag/bench.err; rm -f gpurun_out/r02ag/run_kernel_trace.csv; exit $rc
