#!/bin/bash
# Request-rate counters of the PageRank update kernels (pr_probe.py, RMAT-24 inE, cap) and of
# the gather probe (L2-resident and beyond-L2 8-byte gathers, the request-rate ceiling), one
# rocprofv3 --pmc pass per counter group (slot limits: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM).
# usage: bash scripts/gpu_pmc_pr.sh <tag> [ENV=... for pr_probe]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-pmcpr}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -o $OUT/gather_probe scripts/gather_probe.hip || exit 1
P1="TCP_TCC_READ_REQ_sum TCP_TOTAL_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCC_REQ_sum TCC_BUSY_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  env "$@" PR_PROBE_DEFAULT_ONLY=1 timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/pr$i -o run -- \
      python3 scripts/pr_probe.py 24 20 > $OUT/pr$i.log 2>&1 || { echo "pr pass $i failed"; tail -5 $OUT/pr$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/gp$i -o run -- $OUT/gather_probe \
      > $OUT/gp$i.log 2>&1 || { echo "probe pass $i failed"; tail -5 $OUT/gp$i.log; exit 1; }
  i=$((i+1))
done
python3 scripts/pmc_kernels.py $OUT/pr_counters.json $OUT/pr0 $OUT/pr1 $OUT/pr2
PMC_PER_DISPATCH=1 PMC_KEEP="gather<" python3 scripts/pmc_kernels.py $OUT/probe_counters.json $OUT/gp0 $OUT/gp1 $OUT/gp2
cat $OUT/gp0.log
