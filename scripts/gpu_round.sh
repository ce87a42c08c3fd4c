#!/bin/bash
# Round-closing measurement on one MI355X: the full GPU suite, the plain bench line, the same
# bench under rocprofv3 --kernel-trace --stats, then the PMC traffic passes (gpu_pmc.sh) and
# the partitioned path profiled at world size 1 (gpu_part_prof.sh).
# usage (GPU box): bash scripts/gpu_round.sh <tag>     -> gpurun_out/<tag>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-round}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T -o run -- \
    python3 bench.py > gpurun_out/$T/bench_prof.json 2> gpurun_out/$T/bench_prof.err
rc=$?; echo "prof bench exit $rc"; rm -f gpurun_out/$T/run_kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh ${T}_pmc --rows-scale 0 --sssp-roots 0 || exit 1
bash scripts/gpu_part_prof.sh
