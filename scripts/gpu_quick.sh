TAG=${1:-quick}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; tail -3 gpurun_out/$TAG/bench.err; cat gpurun_out/$TAG/bench.json; exit $rc
