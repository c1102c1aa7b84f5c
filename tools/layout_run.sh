#!/bin/bash
# GPU box: the layout probe's PROBE kinds (tools/layout_probe.hip) and the VA
# arena probe (tools/vmm_arena_probe.cpp), one process each, under gpurun_out/layout/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/layout
timeout -k 10 120 tools/bin/vmm_arena_probe > gpurun_out/layout/arena.jsonl 2>&1 || exit 1
cat gpurun_out/layout/arena.jsonl
for p in ${PROBES:-draw adam collect sgld explore pair}; do
  PROBE=$p TRIALS=${TRIALS:-4} timeout -k 10 240 tools/bin/layout_probe > gpurun_out/layout/$p.jsonl 2>&1 || exit 1
  echo "== $p"; cat gpurun_out/layout/$p.jsonl
done
