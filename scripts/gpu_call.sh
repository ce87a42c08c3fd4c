#!/bin/bash
# Single-source BFS: the bottom-up serial-scan threshold (TGO_BFS_SERIAL) — BFS parity, then
# A/B on RMAT-24 roots.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04za
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py -k "bfs and not multi" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -2 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for v in 32 16 64 128 32 16 64 128; do
    TGO_BFS_SERIAL=$v timeout -k 10 300 python3 scripts/bfs_probe.py 24 8 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/$T/ab.tmp; exit $rc; }
    python3 - "$v" <<'PY' | tee -a gpurun_out/$T/ab.log
import re, sys
g = [float(m.group(1)) for l in open("gpurun_out/r04za/ab.tmp") for m in [re.search(r"GTEPS ([\d.]+)", l)] if m]
print("serial %s: hmean GTEPS %.1f over %d roots" % (sys.argv[1], len(g) / sum(1.0 / x for x in g), len(g)))
PY
done
