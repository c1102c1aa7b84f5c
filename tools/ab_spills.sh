#!/bin/bash
# Round-6 A/B: the library before and after the spill changes (SGLD / SGHMC
# collect instances with per-iteration bases and flags and an un-unrolled slow
# path; Adam GRADONLY scalars per iteration), same process, builds alternating
# (tools/step_ab.py).  Usage: bash tools/ab_spills.sh OLD.so NEW.so
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_spills
libs="$*"
for spec in "resnet101 sgld flat 2,1,1;1,1,1;1,2,1;1,4,1" "resnet101 sghmc flat 2,1,1;1,1,1;1,2,1;1,4,1" \
            "vit_l_32 sgld tensor 1,4,1;2,1,1;1,1,1" "vit_l_32 csghmc flat 1,4,1;1,1,1" \
            "vit_l_32 adam flat 1,4,1;2,4,1"; do
  set -- $spec
  BACKBONE=$1 METHOD=$2 GRAD=$3 ROUNDS=${ROUNDS:-3} GEOMS="$4" COLLECT_ALL=1 timeout -k 10 300 \
    python tools/step_ab.py $libs > gpurun_out/ab_spills/ab_$1_$2_$3.jsonl \
    2> gpurun_out/ab_spills/ab_$1_$2_$3.err || exit $?
  echo "== $1 $2 $3"; grep summary gpurun_out/ab_spills/ab_$1_$2_$3.jsonl
done
