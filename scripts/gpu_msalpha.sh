#!/bin/bash
# Multi-source BFS direction-switch sweep (TGO_MS_ALPHA) with a per-level trace.
# usage (on the GPU box): bash scripts/gpu_msalpha.sh <tag> <alpha>...
TAG=${1:-msalpha}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
for a in "$@"; do
    TGO_TRACE=1 TGO_MS_ALPHA=$a timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --pr-iters 2 --sssp-roots 0 \
        --cpu-baseline 0 > gpurun_out/$TAG/bench_a$a.json 2> gpurun_out/$TAG/bench_a$a.err || exit $?
    echo "alpha $a: $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_a$a.json'));print(d['value'], d['ms_per_step'])")"
done
