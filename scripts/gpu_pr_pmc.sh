#!/bin/bash
# PMC passes over the PageRank update only (pr_probe.py, default variant, RMAT-24): what bounds
# the hot / cold gathers.  One rocprofv3 --pmc pass per counter group, each under its own
# timeout; per-kernel sums in gpurun_out/<tag>/<pass>.csv (scripts/kstats.py style).
# usage: bash scripts/gpu_pr_pmc.sh <tag> [ENV=VAL ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for kv in "$@"; do export "$kv"; done
export PR_PROBE_DEFAULT_ONLY=1
run_pass() {
    local d=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "gather|cold_|fold" --output-format csv \
        -d $OUT/$d -o run -- python3 scripts/pr_probe.py 24 20 > $OUT/$d.log 2>&1
    local rc=$?
    echo "pass $d ($*) exit $rc"
    return $rc
}
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
run_pass tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum && \
run_pass tcc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum && \
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS && \
run_pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in ("tcp", "tcc", "sq", "grbm"):
    tot = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for f in glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
    for k, v in sorted(tot.items()):
        n = max(cnt[(k, c)] for c in v)
        print(d, k, {c: round(x / n) for c, x in v.items()}, "dispatches", n)
PY
