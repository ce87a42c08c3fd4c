#!/bin/bash
# Round-3 call w: the scale-27 one-GPU line with the round-3 code (device assembly + handoff,
# source split), full-size property checks.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r03w; mkdir -p $OUT
TGO_TRACE=1 timeout -k 10 1000 python3 -u scripts/scale27_check.py 27 64 > $OUT/scale27.json 2> $OUT/scale27.log
rc=$?; tail -3 $OUT/scale27.log; cat $OUT/scale27.json; exit $rc
