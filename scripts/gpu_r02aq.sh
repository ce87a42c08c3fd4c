#!/bin/bash
# rocprof kernel summary of the default bench with the committed defaults.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02aq
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02aq -o run -- \
    python3 bench.py > gpurun_out/r02aq/bench_prof.json 2> gpurun_out/r02aq/bench_prof.err
rc=$?; echo "prof bench exit $rc"; rm -f gpurun_out/r02aq/run_kernel_trace.csv; exit $rc
