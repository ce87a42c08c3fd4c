#!/bin/bash
# PageRank tile size probe: the default library (kTile 4096) against a TGO_KTILE=2048 build
# (make -C titan_amd/csrc OUT=../libtitan_gpu_olap_t2048.so OBJDIR=build_t2048 EXTRA=-DTGO_KTILE=2048).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ktile
for lib in titan_amd/libtitan_gpu_olap.so titan_amd/libtitan_gpu_olap_t2048.so titan_amd/libtitan_gpu_olap.so; do
  TGO_LIB_PATH=$PWD/$lib PR_PROBE_DEFAULT_ONLY=1 timeout -k 10 300 python3 scripts/pr_probe.py 24 20 \
      > gpurun_out/ktile/probe.log 2>&1 || { tail -5 gpurun_out/ktile/probe.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ktile/probe.log)"
done
