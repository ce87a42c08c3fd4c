#!/bin/bash
# Delta SSSP: pipelined stop checks (host-mapped publish per batch) — parity, then A/B with
# the batch size.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=r04x
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_trace.py -k "sssp or delta or config5 or trace" > gpurun_out/$T/parity.log 2>&1
rc=$?; tail -3 gpurun_out/$T/parity.log; [ $rc -eq 0 ] || exit $rc
for v in "TGO_DS_PIPE=0" "TGO_DS_PIPE=1" "TGO_DS_BATCH=16" "TGO_DS_BATCH=4" "TGO_DS_PIPE=0" "TGO_DS_PIPE=1" "TGO_DS_BATCH=16" "TGO_DS_BATCH=4"; do
    env $v timeout -k 10 300 python3 scripts/sssp_once.py 24 4 > gpurun_out/$T/ab.tmp 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/$T/ab.tmp; exit $rc; }
    grep "GTEPS" gpurun_out/$T/ab.tmp | sed "s/^/$v: /" >> gpurun_out/$T/ab.log
done
python3 - <<'PY'
import re, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r04x/ab.log"):
    m = re.match(r"(\S+): .*kernel ([\d.]+) ms", l)
    if m: d[m.group(1)].append(float(m.group(2)))
for k, v in d.items(): print(k, len(v), round(sum(v) / len(v), 3))
PY
