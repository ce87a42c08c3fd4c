#!/bin/bash
# Round-close evidence in one call: the full GPU suite and smoke, the bench line under
# rocprofv3 --kernel-trace --stats, and the PMC traffic passes.  OUT tag: $1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-close}
bash scripts/gpu_tests.sh $T tests -m gpu || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || exit 1
bash scripts/gpu_measure.sh ${T}m || exit 1
bash scripts/gpu_pmc.sh ${T}pmc
