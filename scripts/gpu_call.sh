#!/bin/bash
# Single-source BFS with the 128-entry serial scan by default: BFS parity, A/B of larger
# thresholds, the bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04zb
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_scale27.py tests/test_gpu_distributed.py -k "bfs and not multi" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -2 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for v in 128 256 512 1024 128 256 512 1024; do
    TGO_BFS_SERIAL=$v timeout -k 10 300 python3 scripts/bfs_probe.py 24 8 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/$T/ab.tmp; exit $rc; }
    python3 - "$v" <<'PY' | tee -a gpurun_out/$T/ab.log
import re, sys
g = [float(m.group(1)) for l in open("gpurun_out/r04zb/ab.tmp") for m in [re.search(r"GTEPS ([\d.]+)", l)] if m]
print("serial %s: hmean GTEPS %.1f over %d roots" % (sys.argv[1], len(g) / sum(1.0 / x for x in g), len(g)))
PY
done
timeout -k 10 500 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; cut -c1-300 gpurun_out/$T/bench.json; exit $rc
