cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02ad
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "multi" --timeout 120 --timeout-method thread > gpurun_out/r02ad/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r02ad/tests.log; [ $rc -eq 0 ] || exit $rc
for f in 0 1; do
  TGO_MS_FILTER=$f timeout -k 10 300 python3 bench.py --steps 3 --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 > gpurun_out/r02ad/bench_f$f.json 2> gpurun_out/r02ad/bench_f$f.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r02ad/bench_f$f.json'));print($f, d['value'], d['ms_per_step'], d['roofline_bfs']['achieved'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02ad -o tr -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 > /dev/null 2>&1
echo prof $?
