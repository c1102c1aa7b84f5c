#!/bin/bash
# Placement A/B (tooling): the default bench with the swept vectors built from
# 1 GiB chunks (ViT-L/32: two per vector) vs one chunk per vector
# (BDL_CHUNK_MB=2048), alternating processes on one box.
mkdir -p gpurun_out
for i in 1 2 3; do
  for mb in 1024 2048; do
    BDL_CHUNK_MB=$mb timeout -k 10 200 python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-aux \
      > gpurun_out/chunk_${mb}_$i.json 2>/dev/null || exit 1
  done
done
