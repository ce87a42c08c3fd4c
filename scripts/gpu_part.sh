#!/bin/bash
# Partitioned-path check on one GPU: parity tests, then bench.py --partitioned (world size 1,
# NCCL) with and without the degree-grouped device layout.
TAG=${1:-part}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for lay in ${LAYOUTS:-1 0}; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --partitioned --steps 2 --warmup 1 --layout $lay "$@" \
      > gpurun_out/$TAG/bench_part_l$lay.json 2> gpurun_out/$TAG/bench_part_l$lay.err
  rc=$?; echo "layout $lay exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/$TAG/bench_part_l$lay.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/bench_part_l$lay.json')); print('GTEPS', d['value'], 'PR s/it', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'], 'sssp', d['sssp'])"
done
