#!/bin/bash
# A/B of the placement search's initial chunk pool: the default (roles x per +
# 2 x per chunks, more only while no fast pair shows) vs BDL_PLACEMENT_SPARE
# spare chunks from the start, alternating fresh bench processes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/spare_ab.jsonl
: > $OUT
for i in $(seq 1 ${ROUNDS:-4}); do
  for sp in 0 ${SPARE:-12}; do
    BDL_PLACEMENT_SPARE=$sp timeout -k 10 200 python bench.py --no-aux --no-cpu-baseline \
      --e2e-steps 0 > gpurun_out/spare_ab_run.json 2> gpurun_out/spare_ab_run.err || exit 1
    python3 - "$sp" "$i" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/spare_ab_run.json"))
p = d["placement"]
print(json.dumps({"spare": int(sys.argv[1]), "round": int(sys.argv[2]),
                  "kernel_ms": d["kernels"]["explore"]["avg_ms"], "value": d["value"],
                  "chosen_ms": p.get("chosen_ms"), "kept": p.get("kept"),
                  "search_s": p.get("search_seconds", p.get("seconds")),
                  "pairs_timed": p.get("pairs_timed"), "chunks": p.get("chunks_allocated")}))
PY
    tail -1 $OUT
  done
done
