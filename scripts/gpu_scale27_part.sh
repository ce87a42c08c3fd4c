#!/bin/bash
# Scale-27 one-GPU re-measure (scale27_check.py) and the world-1 partitioned bench profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-s27}
mkdir -p gpurun_out/$T
timeout -k 10 700 python3 -u scripts/scale27_check.py > gpurun_out/$T/scale27.json 2> gpurun_out/$T/scale27.log
rc=$?; echo "scale27 exit $rc"; grep -E "\[scale27\]|device loop" gpurun_out/$T/scale27.log | tail -12; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_part_prof.sh && cp -r gpurun_out/partprof gpurun_out/$T/
