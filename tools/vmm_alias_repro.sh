#!/bin/bash
# Every scenario of tools/vmm_alias_repro.cpp in its own process, at two chunk
# sizes; one JSON line each.  Output: gpurun_out/vmm_alias_repro.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/vmm_alias_repro.jsonl
: > $out
for mb in 64 586; do
  for sc in free_reuse free_reuse_sync per_chunk_free remap_in_place fresh_range late_views after_hipfree arena; do
    timeout -k 5 60 ./tools/bin/vmm_alias_repro $sc $mb >> $out 2>&1 || { echo "rc=$? at $sc $mb"; exit 1; }
  done
done
cat $out
