#!/bin/bash
# A/B of PageRank gather variants on RMAT-24 (pr_probe.py, default path): ms/update per
# variant and a digest of the ranks, compared bitwise with the first variant.
# usage: bash scripts/gpu_pr_ab.sh <tag> "ENV=.. ENV=.." "ENV=.." ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for v in "$@"; do
  env $v PR_PROBE_DEFAULT_ONLY=1 PR_PROBE_SAVE=$OUT/pr$i.sha timeout -k 10 300 \
      python3 scripts/pr_probe.py 24 20 > $OUT/probe$i.log 2>&1 || { tail -5 $OUT/probe$i.log; exit 1; }
  same=$(cmp -s $OUT/pr0.sha $OUT/pr$i.sha && echo True || echo False)
  echo "[$v] bitwise_equal_first=$same $(tail -1 $OUT/probe$i.log)"
  i=$((i+1))
done
