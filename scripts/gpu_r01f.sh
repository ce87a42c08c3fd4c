cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r01f
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01f/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r01f/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./scripts/gather_probe > gpurun_out/r01f/gather_probe.log 2>&1; rc=$?; cat gpurun_out/r01f/gather_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/sssp_probe.py 24 0,32,64,128,256,512,2048 > gpurun_out/r01f/sssp_probe.log 2>&1; rc=$?; cat gpurun_out/r01f/sssp_probe.log; exit $rc
