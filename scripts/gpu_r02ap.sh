#!/bin/bash
# PMC traffic with the 384 K hot head, then the partitioned world-1 bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_pmc.sh r02ap_pmc --rows-scale 0 --sssp-roots 0 || exit 1
mkdir -p gpurun_out/r02ap
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29539
timeout -k 10 400 python3 bench.py --partitioned --steps 5 --warmup 2 --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 \
    > gpurun_out/r02ap/bench_part.json 2> gpurun_out/r02ap/bench_part.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r02ap/bench_part.json')); print('part GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'])"
