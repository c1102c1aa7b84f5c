#!/bin/bash
# Round-6 A/B: the depth-1 cSGHMC collect / init instances with SGPR-held
# Philox inputs (flavor -DBDL_HELD_CSG) vs re-read per call, same process,
# builds alternating (tools/step_ab.py: explore, Welford collect and init at
# every geometry, flat and per-tensor gradients); the flag lived in bdl_kernels.hpp for this
# A/B only (not adopted: within 0.5 %, profiles/round6/ab_held_csg/).  Usage: bash tools/ab_held_csg.sh A.so B.so
set -u
LIB_A=$1
LIB_B=$2
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_held_csg
for g in flat tensor; do
  BACKBONE=vit_l_32 METHOD=csghmc GRAD=$g ROUNDS=3 GEOMS="1,1,1;2,1,1;1,4,1" COLLECT_ALL=1 INIT=1 \
    timeout -k 10 400 python tools/step_ab.py "$LIB_A" "$LIB_B" \
    > gpurun_out/ab_held_csg/ab_$g.jsonl 2> gpurun_out/ab_held_csg/ab_$g.err || exit $?
  echo "== $g"; grep summary gpurun_out/ab_held_csg/ab_$g.jsonl
done
