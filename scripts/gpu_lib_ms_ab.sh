#!/bin/bash
# A/B of library builds on the multi-source BFS probe (ms_probe.py, RMAT-24 bothE, 64 roots),
# interleaved; the reached / entries totals must agree (the same traversal).
# usage: bash scripts/gpu_lib_ms_ab.sh <tag> <rounds> lib1.so lib2.so ...   (ENV via MS_AB_ENV)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    env TGO_LIB_PATH=$PWD/$lib $MS_AB_ENV timeout -k 10 200 python3 scripts/ms_probe.py 24 5 > $OUT/ms.log 2>&1 || { tail -5 $OUT/ms.log; exit 1; }
    echo "$lib $(grep msbfs $OUT/ms.log)" | tee -a $OUT/ab.log
  done
done
