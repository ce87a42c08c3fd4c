#!/bin/bash
# Partitioned path at world size 1 on one GPU, profiled: where the multi-source sweep and the
# single-source levels spend their time next to the one-GPU path.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/partprof
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/partprof -o run -- \
    python3 bench.py --partitioned --steps 2 --warmup 1 --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 \
    > gpurun_out/partprof/bench.json 2> gpurun_out/partprof/bench.err
rc=$?; echo "exit $rc"; tail -3 gpurun_out/partprof/bench.err
python3 -c "import json; d=json.load(open('gpurun_out/partprof/bench.json')); print('GTEPS', d['value'], 'PR', d['pagerank_s_per_iter'], 'ss', d['single_source_gteps_hmean'])"
exit $rc
