#!/bin/bash
# A/B of library builds on the PageRank probe (RMAT-24, default path), interleaved; each
# build's ranks digest goes to <tag>/<lib>.sha (builds that must agree bit for bit).
# usage: bash scripts/gpu_lib_ab.sh <tag> <rounds> lib1.so lib2.so ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    TGO_LIB_PATH=$PWD/$lib PR_PROBE_DEFAULT_ONLY=1 PR_PROBE_SAVE=$OUT/$(basename $lib .so).sha \
        timeout -k 10 300 python3 scripts/pr_probe.py 24 20 > $OUT/probe.log 2>&1 || { tail -5 $OUT/probe.log; exit 1; }
    echo "$lib $(tail -1 $OUT/probe.log)" | tee -a $OUT/ab.log
  done
done
md5sum $OUT/*.sha | tee -a $OUT/ab.log
