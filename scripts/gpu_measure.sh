#!/bin/bash
# One measurement call: the Java multi-GPU natives at world 1 (JNI harness), the plain bench
# line and the same bench under rocprofv3 --kernel-trace --stats.
# usage (GPU box): bash scripts/gpu_measure.sh <tag>     -> gpurun_out/<tag>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-measure}
mkdir -p gpurun_out/$T
timeout -k 10 240 python -u -m pytest tests/test_jni_shim.py -m gpu -q --timeout 200 --timeout-method thread \
    > gpurun_out/$T/jni_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/$T/jni_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T -o run -- \
    python3 bench.py > gpurun_out/$T/bench_prof.json 2> gpurun_out/$T/bench_prof.err
rc=$?; echo "prof bench exit $rc"; rm -f gpurun_out/$T/run_kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py gpurun_out/$T/run_kernel_stats.csv 14
