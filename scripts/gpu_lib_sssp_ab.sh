#!/bin/bash
# A/B of library builds on the weighted RMAT-24 delta SSSP probe (sssp_once.py, 4 roots),
# interleaved: kernel ms per root and GTEPS.  usage: bash scripts/gpu_lib_sssp_ab.sh <tag> <rounds> lib.so[:ENV=..] ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    lib=${spec%%:*}; ev=""; [ "$spec" != "$lib" ] && ev=${spec#*:}
    env TGO_LIB_PATH=$PWD/$lib $ev timeout -k 10 200 python3 scripts/sssp_once.py 24 4 > $OUT/sssp.log 2>&1 || { tail -5 $OUT/sssp.log; exit 1; }
    echo "$spec $(grep -o 'kernel [0-9.]* ms' $OUT/sssp.log | tr '\n' ' ') $(grep -o 'GTEPS(kernel) [0-9.]*' $OUT/sssp.log | tr '\n' ' ')" | tee -a $OUT/ab.log
  done
done
