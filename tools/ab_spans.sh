#!/bin/bash
# Round-6 probe: the cSGHMC explore / Welford collect / Welford init at
# grid-stride (x,y,1) vs contiguous per-block spans (x,y,0), production build,
# same process (tools/step_ab.py COLLECT_ALL=1 INIT=1).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_spans
for g in flat tensor; do
  BACKBONE=vit_l_32 METHOD=csghmc GRAD=$g ROUNDS=3 GEOMS="1,1,1;1,1,0;2,1,1;2,1,0;1,4,1;1,4,0;1,2,0" \
    COLLECT_ALL=1 INIT=1 timeout -k 10 400 python tools/step_ab.py bayesdll_amd/libbdl_sgmcmc.so \
    > gpurun_out/ab_spans/ab_$g.jsonl 2> gpurun_out/ab_spans/ab_$g.err || exit $?
  echo "== $g"; grep summary gpurun_out/ab_spans/ab_$g.jsonl
done
