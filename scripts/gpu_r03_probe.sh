#!/bin/bash
# Round-3 probe call: new GPU tests (args), multi-source BFS level trace + per-kernel trace of
# one sweep, PageRank tile A/B, PageRank PMC passes.
# usage: bash scripts/gpu_r03_probe.sh <tag> "<pytest args or empty>"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; TESTS=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -4 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
TGO_TRACE=1 timeout -k 10 300 python3 scripts/ms_probe.py 24 3 > $OUT/ms_probe.log 2>&1 || { tail -5 $OUT/ms_probe.log; exit 1; }
grep -v "assemble" $OUT/ms_probe.log | tail -14
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/mstrace -o run -- python3 scripts/ms_probe.py 24 1 \
    > $OUT/ms_trace.log 2>&1 || { tail -5 $OUT/ms_trace.log; exit 1; }
python3 - $OUT/mstrace <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ms = [r for r in rows if "ms_" in r["Kernel_Name"] or "scan" in r["Kernel_Name"].lower() or "publish" in r["Kernel_Name"]]
# the last sweep: from the last ms_seed on
last = max(i for i, r in enumerate(ms) if "ms_seed" in r["Kernel_Name"])
t0 = int(ms[last]["Start_Timestamp"])
for r in ms[last:]:
    if "ms_reach" in r["Kernel_Name"] or "ms_extract" in r["Kernel_Name"]:
        break
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  {r['Kernel_Name'][:60]}")
PY
rm -rf $OUT/mstrace
bash scripts/gpu_pr_ab.sh $TAG/ab "TGO_PR_X=0" "TGO_PR_HOT_TILE=8192" "TGO_PR_HOT_TILE=16384" \
    "TGO_PR_HOT_TILE=8192 TGO_PR_HOT_PIPE=1" "TGO_PR_HOT_TILE=16384 TGO_PR_HOT_PIPE=1" || exit 1
bash scripts/gpu_pr_pmc.sh $TAG/pmc
