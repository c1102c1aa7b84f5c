#!/bin/bash
# Placement A/B (tooling): the default bench with 3 plain torch allocations
# competing with the chunk composites (BDL_PLACEMENT_TORCH=0: 3 pairings, the
# round-2 first version) vs 5 (the default: 10 pairings), alternating
# processes on one box.
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for t in 0 2; do
    BDL_PLACEMENT_TORCH=$t timeout -k 10 200 python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-aux \
      > gpurun_out/tcand_${t}_$i.json 2>/dev/null || exit 1
  done
done
