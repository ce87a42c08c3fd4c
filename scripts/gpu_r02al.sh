#!/bin/bash
# Touched-chunk pack skipping: distributed GPU tests, then the partitioned world-1 bench twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02al
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r02al/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r02al/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29537
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --partitioned --steps 5 --warmup 2 --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 \
      > gpurun_out/r02al/bench_part_$i.json 2> gpurun_out/r02al/bench_part_$i.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r02al/bench_part_$i.json')); print('run $i GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'])"
done
