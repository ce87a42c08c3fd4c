#!/bin/bash
# Fixed-point hot pass: E sweep (pr_probe.py) + a kernel trace of the default (pr_probe, one variant).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-prfx}
OUT=gpurun_out/$TAG; mkdir -p $OUT
PR_PROBE_VARIANTS=${PR_PROBE_VARIANTS:-'[{"TGO_PR_FX": "1", "TGO_PR_FX_E": "262144"}, {"TGO_PR_FX": "1", "TGO_PR_FX_E": "524288"}, {"TGO_PR_FX": "1", "TGO_PR_FX_E": "1048576"}]'} \
  timeout -k 10 300 python3 -u scripts/pr_probe.py 24 20 > $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
cat $OUT/probe.log
PV='[{}]'; [ -n "$FX_E" ] && PV='[{"TGO_PR_FX_E": "'$FX_E'"}]'
PR_PROBE_VARIANTS=$PV timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 scripts/pr_probe.py 24 20 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
rm -f $OUT/prof/run_kernel_trace.csv
python3 scripts/kstats.py $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -20 || head -15 $OUT/prof/run_kernel_stats.csv
