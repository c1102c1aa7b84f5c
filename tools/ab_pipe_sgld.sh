#!/bin/bash
# Round-6 A/B: a software-pipelined plain SGLD sweep (flavours built with
# -DBDL_PIPE_SGLD=<depth> [-DBDL_PIPE_SGLD_HELD]) against production, same
# process, builds alternating (tools/step_ab.py).  The flavour code lived in
# bdl_kernels.hpp for this A/B only: pipelined, the sweep ran 0.3385 vs 0.2436 ms
# at 1 x 1 and 0.2029 vs 0.1693 at 2 x 1 (ResNet-101; profiles/round6/ab_pipe_sgld/),
# as round 4 found.  Usage: bash tools/ab_pipe_sgld.sh LIB...
set -u
LIBS=("$@")
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_pipe_sgld
for spec in "resnet101 flat" "vit_l_32 tensor"; do
  set -- $spec
  BACKBONE=$1 METHOD=sgld GRAD=$2 ROUNDS=3 GEOMS="1,1,1;2,1,1;1,2,1;1,4,1" \
    timeout -k 10 300 python tools/step_ab.py "${LIBS[@]}" \
    > gpurun_out/ab_pipe_sgld/ab_$1.jsonl 2> gpurun_out/ab_pipe_sgld/ab_$1.err || exit $?
  echo "== $1 $2"; grep summary gpurun_out/ab_pipe_sgld/ab_$1.jsonl | grep '"sgld"'
done
