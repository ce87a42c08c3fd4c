#!/bin/bash
# A/B of delta-stepping variants on the bench's weighted RMAT-24 inE graph (sssp_once.py, 4
# giant-component roots, one process per variant): kernel ms per root and GTEPS.
# usage: bash scripts/gpu_sssp_ab.sh <tag> "ENV=.. ENV=.." "ENV=.." ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for v in "$@"; do
  env $v timeout -k 10 200 python3 scripts/sssp_once.py 24 4 > $OUT/sssp$i.log 2>&1 || { tail -5 $OUT/sssp$i.log; exit 1; }
  echo "[$v] $(grep -o 'kernel [0-9.]* ms' $OUT/sssp$i.log | tr '\n' ' ') $(grep -o 'GTEPS(kernel) [0-9.]*' $OUT/sssp$i.log | tr '\n' ' ')"
  i=$((i+1))
done
