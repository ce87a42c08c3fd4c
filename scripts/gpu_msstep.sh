#!/bin/bash
# MS-BFS pull round-trip width A/B (TGO_MS_STEP 4 / 8 / 16): bench value, no CPU baseline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/msstep
for st in 8 16 4; do
  TGO_MS_STEP=$st timeout -k 10 300 python3 bench.py --steps 3 --cpu-baseline 0 --rows-scale 0 --sssp-roots 0 --pr-iters 2 \
      > gpurun_out/msstep/bench_$st.json 2> gpurun_out/msstep/bench_$st.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/msstep/bench_$st.json'));print('step $st', d['value'], d['validation'])"
done
