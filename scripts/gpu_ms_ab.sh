#!/bin/bash
# A/B of multi-source BFS variants on the bench graph (ms_probe.py, RMAT-24 bothE, 64 roots):
# ms/sweep, GTEPS and the reached / entries totals (equal across variants = same traversal).
# usage: bash scripts/gpu_ms_ab.sh <tag> "ENV=.. ENV=.." "ENV=.." ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for v in "$@"; do
  env $v timeout -k 10 200 python3 scripts/ms_probe.py 24 5 > $OUT/ms$i.log 2>&1 || { tail -5 $OUT/ms$i.log; exit 1; }
  echo "[$v] $(grep msbfs $OUT/ms$i.log)"
  i=$((i+1))
done
