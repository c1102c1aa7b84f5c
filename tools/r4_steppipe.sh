#!/bin/bash
# Round-4 GPU box: pipelined step sweep (tools/bin/libbdl_steppipe.so) vs the
# production build, SGLD on ResNet-101 and ViT-L/32, one process each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
for bb in resnet101 vit_l_32; do
  BACKBONE=$bb METHOD=sgld ROUNDS=3 GEOMS="1,1,1;1,2,1;1,4,1;2,1,1;2,4,1;3,4,1" timeout -k 10 400 \
    python tools/step_ab.py bayesdll_amd/libbdl_sgmcmc.so tools/bin/libbdl_steppipe.so \
    > gpurun_out/r4/steppipe_$bb.jsonl 2> gpurun_out/r4/steppipe_$bb.err || exit $?
  echo "== $bb"; grep summary gpurun_out/r4/steppipe_$bb.jsonl
done
