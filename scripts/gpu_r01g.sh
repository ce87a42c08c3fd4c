#!/bin/bash
# Round-1 check: parity tests, default bench under rocprofv3 --stats, then the partitioned
# path at world size 1 (NCCL) with its SSSP leg.
TAG=${1:-r01g}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
bash scripts/gpu_check.sh $TAG || exit $?
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --partitioned --steps 2 --warmup 1 > gpurun_out/$TAG/bench_part.json 2> gpurun_out/$TAG/bench_part.err
rc=$?; echo "partitioned exit $rc"; tail -3 gpurun_out/$TAG/bench_part.err; cat gpurun_out/$TAG/bench_part.json; exit $rc
