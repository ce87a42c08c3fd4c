#!/bin/bash
# Partitioned world-1 bench (no profiler), fixed-capacity sparse exchange on vs off.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/partab
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535
for fb in 67108864 0 67108864; do
  TGO_MS_FIXED_BYTES=$fb timeout -k 10 400 python3 bench.py --partitioned --steps 5 --warmup 2 --cpu-baseline 0 \
      --rows-scale 0 --sssp-roots 0 > gpurun_out/partab/bench_$fb.json 2> gpurun_out/partab/bench_$fb.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/partab/bench_$fb.json')); print('fixed_bytes $fb GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'])"
done
