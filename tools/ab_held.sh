#!/bin/bash
# Round-6 A/B: the depth-1 SGLD / SGHMC sweeps drawing their Philox noise from
# generator inputs held in SGPRs (flavor built with -DBDL_HELD_NOISE_U1, the
# A/B flag; adopted for the collect instances as chunk_fast's kHeldNoise) vs
# re-read per call.  Same process, builds alternating (tools/step_ab.py),
# collects at every geometry.  Usage: bash tools/ab_held.sh BASE.so OTHER.so
set -u
LIB_A=$1
LIB_B=$2
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_held
for spec in "resnet101 sgld flat" "resnet101 sghmc flat" "vit_l_32 sgld tensor"; do
  set -- $spec
  BACKBONE=$1 METHOD=$2 GRAD=$3 ROUNDS=3 GEOMS="1,1,1;2,1,1;1,4,1" COLLECT_ALL=1 \
    timeout -k 10 300 python tools/step_ab.py "$LIB_A" "$LIB_B" \
    > gpurun_out/ab_held/ab_$1_$2_$3.jsonl 2> gpurun_out/ab_held/ab_$1_$2_$3.err || exit $?
  echo "== $1 $2 $3"; grep summary gpurun_out/ab_held/ab_$1_$2_$3.jsonl
done
