#!/bin/bash
# Partitioned SSSP protocol check: the native driver tests (in-process worlds 2 / 4 at RMAT-24
# and the small distributed cases), then the world-1 probe (plain and under rocprofv3
# --kernel-trace) for the per-phase timeline.  OUT=gpurun_out/<tag>
set -o pipefail
OUT=${OUT:-gpurun_out/part_sssp}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_gpu_distributed.py -k "sssp or native" -m gpu > "$OUT/tests.log" 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 360 --timeout-method thread \
    tests/test_gpu_fullsize.py -k "config5" -m gpu >> "$OUT/tests.log" 2>&1 &&
timeout -k 10 240 python -u scripts/part_sssp_probe.py 24 2 > "$OUT/probe.log" 2>&1 &&
if [ -n "$AB_ENV" ]; then env $AB_ENV timeout -k 10 240 python -u scripts/part_sssp_probe.py 24 2 > "$OUT/probe_ab.log" 2>&1; fi &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u scripts/part_sssp_probe.py 24 1 \
    > "$OUT/probe_prof.log" 2>&1
