#!/bin/bash
# Round-2 closing measurement: full GPU suite, plain bench, rocprof-profiled bench, PMC traffic.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r02final}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T -o run -- \
    python3 bench.py > gpurun_out/$T/bench_prof.json 2> gpurun_out/$T/bench_prof.err
rc=$?; echo "prof bench exit $rc"; rm -f gpurun_out/$T/run_kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh ${T}_pmc --rows-scale 0 --sssp-roots 0
bash scripts/gpu_part_prof.sh
