#!/bin/bash
# HBM traffic of the bench's dominant kernels from PMC counters, one rocprofv3 pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950's 4 TCC slots).
# usage (on the GPU box): bash scripts/gpu_pmc.sh <tag> [bench args...]
# writes gpurun_out/<tag>/pmc_traffic.json (copy it to profiles/ to have bench.py report it)
TAG=${1:-pmc}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
run_pass() {   # $1 = dir name, rest = counters
    local d=$1; shift
    timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$d -o run -- \
        python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 $BENCH_ARGS > $OUT/$d.log 2>&1
    local rc=$?
    echo "pass $d ($*) exit $rc"
    return $rc
}
BENCH_ARGS="$*"
# req: the request-rate set of DESIGN §4 (L2 requests, L2 channel / TA busy cycles) — the
# bound of the PageRank and multi-source gathers is the L2 request rate, not HBM bytes
run_pass fetch FETCH_SIZE && run_pass write WRITE_SIZE && run_pass hit TCC_HIT_sum TCC_MISS_sum && \
    run_pass ea TCC_EA0_RDREQ_sum && \
    run_pass req TCC_REQ_sum TCC_BUSY_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE || exit 1
python3 scripts/pmc_traffic.py $OUT/pmc_traffic.json $OUT/fetch $OUT/write $OUT/hit $OUT/ea $OUT/req
