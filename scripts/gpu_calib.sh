#!/bin/bash
# PMC calibration on known byte counts (scripts/pmc_calib.hip) + the same counters on the
# PageRank update of the bench graph.  usage (GPU box): bash scripts/gpu_calib.sh <tag>
TAG=${1:-calib}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || echo "list failed"
timeout -k 5 60 ./scripts/pmc_calib > $OUT/calib_plain.log 2>&1 || { echo "plain run failed"; exit 1; }
cat $OUT/calib_plain.log
pass() {   # $1 = name, $2 = program tag, rest = counters
    local d=$1 prog=$2; shift 2
    if [ "$prog" = calib ]; then
        timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$d -o run -- ./scripts/pmc_calib > $OUT/$d.log 2>&1
    else
        PR_PROBE_DEFAULT_ONLY=1 timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$d -o run -- python3 scripts/pr_probe.py 24 4 > $OUT/$d.log 2>&1
    fi
    local rc=$?; echo "pass $d ($*) exit $rc"; return $rc
}
pass c_fetch calib FETCH_SIZE && pass c_write calib WRITE_SIZE && pass c_hit calib TCC_HIT_sum TCC_MISS_sum && \
pass c_ea calib TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum && \
pass p_fetch pr FETCH_SIZE && pass p_write pr WRITE_SIZE && pass p_hit pr TCC_HIT_sum TCC_MISS_sum && \
pass p_ea pr TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
