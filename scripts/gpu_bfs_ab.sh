#!/bin/bash
# A/B of single-source BFS variants (bfs_probe.py, RMAT-24 bothE, ROOTS roots, default 8): per-root GTEPS and
# their harmonic mean per variant.
# usage: bash scripts/gpu_bfs_ab.sh <tag> "ENV=.. ENV=.." "ENV=.." ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for v in "$@"; do
  env $v timeout -k 10 200 python3 scripts/bfs_probe.py ${SCALE:-24} ${ROOTS:-8} > $OUT/bfs$i.log 2>&1 || { tail -5 $OUT/bfs$i.log; exit 1; }
  echo "[$v] $(python3 -c "
import re,sys
g=[float(x) for x in re.findall(r'GTEPS ([0-9.]+)', open('$OUT/bfs$i.log').read())]
print('hmean %.1f GTEPS over %d roots:' % (len(g)/sum(1/x for x in g), len(g)), ' '.join('%.0f' % x for x in g))")"
  i=$((i+1))
done
