#!/bin/bash
# Pull-shape sweeps equal (new test), SSSP with non-returning far pending atomics (parity +
# per-root times), then split budget / direction switch A/B with the 64-entry trips.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04z9
mkdir -p gpurun_out/$T
timeout -k 10 800 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py -k "pull_shapes or settle_sums or sssp or delta or config5" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    timeout -k 10 300 python3 scripts/sssp_once.py 24 4 > gpurun_out/$T/ss.tmp 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/$T/ss.tmp; exit $rc; }
    grep GTEPS gpurun_out/$T/ss.tmp >> gpurun_out/$T/sssp.log
done
python3 - <<'PY'
import re
v = [float(m.group(1)) for l in open("gpurun_out/r04z9/sssp.log") for m in [re.search(r"kernel ([\d.]+) ms", l)] if m]
print("sssp kernel ms per root: mean %.3f over %d" % (sum(v) / len(v), len(v)))
PY
for v in "TGO_MS_SPLIT=0.005" "TGO_MS_SPLIT=0" "TGO_MS_SPLIT=0.002" "TGO_MS_SPLIT=0.01" "TGO_MS_SPLIT=0.02" \
         "TGO_MS_ALPHA=8" "TGO_MS_ALPHA=16" "TGO_MS_ALPHA=24" \
         "TGO_MS_SPLIT=0.005" "TGO_MS_SPLIT=0" "TGO_MS_SPLIT=0.002" "TGO_MS_SPLIT=0.01" "TGO_MS_SPLIT=0.02" \
         "TGO_MS_ALPHA=8" "TGO_MS_ALPHA=16" "TGO_MS_ALPHA=24"; do
    env $v timeout -k 10 300 python3 scripts/ms_probe.py 24 5 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; echo "$v: $(tail -1 gpurun_out/$T/ab.tmp)" | cut -c1-110 | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
done
