#!/bin/bash
# Round-4 close, part B: the bench under rocprofv3 --kernel-trace --stats (the same command as
# the bench line), then the PMC passes (traffic + the request-rate set) of gpu_pmc.sh.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04f}
mkdir -p gpurun_out/$T
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T -o run -- \
    python3 bench.py > gpurun_out/$T/bench_prof.json 2> gpurun_out/$T/bench_prof.err
rc=$?; echo "prof bench exit $rc"; rm -f gpurun_out/$T/run_kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py gpurun_out/$T/run_kernel_stats.csv 14
bash scripts/gpu_pmc.sh ${T}_pmc --rows-scale 0 --sssp-roots 0
