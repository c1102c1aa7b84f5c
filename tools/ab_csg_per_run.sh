#!/bin/bash
# Round-6 A/B: the depth-1 cSGHMC collect / init instances on the plain
# sweep's per-run loop (flavour -DBDL_CSG_COLLECT_PER_RUN=1) vs the
# per-iteration run lookup, same process, builds alternating (tools/step_ab.py).
# The flag lived in bdl_kernels.hpp for the A/B; adopted for the init kinds
# (csg_collect_per_run).  Usage: bash tools/ab_csg_per_run.sh A.so B.so
set -u
LIB_A=$1
LIB_B=$2
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_csg_per_run
for g in flat tensor; do
  BACKBONE=vit_l_32 METHOD=csghmc GRAD=$g ROUNDS=4 GEOMS="1,1,1;2,1,1;3,1,1" COLLECT_ALL=1 INIT=1 \
    timeout -k 10 400 python tools/step_ab.py "$LIB_A" "$LIB_B" \
    > gpurun_out/ab_csg_per_run/ab_$g.jsonl 2> gpurun_out/ab_csg_per_run/ab_$g.err || exit $?
  echo "== $g"; grep summary gpurun_out/ab_csg_per_run/ab_$g.jsonl
done
