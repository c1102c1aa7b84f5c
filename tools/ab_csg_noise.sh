#!/bin/bash
# Round-6 A/B: where the cSGHMC collect steps (Welford init / steady) draw
# their Philox noise relative to the loads — production vs the gradient loaded
# through the global address space (F=gv, -DBDL_CSG_COLLECT_GVLOAD) vs the
# Philox inputs waited for before the vector loads (F=pf,
# -DBDL_CSG_PHILOX_FIRST) — same process, builds alternating (tools/step_ab.py).
# Both macros lived in bdl_kernels.hpp for this A/B only (not adopted, not
# committed); results in profiles/round6/ab_csg_noise/.
# Usage: bash tools/ab_csg_noise.sh LIB [LIB ...]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_csg_noise
for g in flat tensor; do
  BACKBONE=vit_l_32 METHOD=csghmc GRAD=$g ROUNDS=${ROUNDS:-3} GEOMS="1,1,1;2,1,1;1,4,1" \
    COLLECT_ALL=1 INIT=1 timeout -k 10 400 python tools/step_ab.py "$@" \
    > gpurun_out/ab_csg_noise/ab_$g.jsonl 2> gpurun_out/ab_csg_noise/ab_$g.err || exit $?
  echo "== $g"; grep summary gpurun_out/ab_csg_noise/ab_$g.jsonl
done
