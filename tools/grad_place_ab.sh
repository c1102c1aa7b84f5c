#!/bin/bash
# A/B of placing the flat gradient with the set (BDL_PLACEMENT_GRAD=0 vs 1),
# alternating fresh bench processes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/grad_place_ab.jsonl
: > $OUT
for i in $(seq 1 ${ROUNDS:-6}); do
  for rt in 0 1; do
    BDL_PLACEMENT_GRAD=$rt timeout -k 10 200 python bench.py --no-aux --no-cpu-baseline \
      --e2e-steps 0 > gpurun_out/grad_place_ab_run.json 2> gpurun_out/grad_place_ab_run.err || exit 1
    python3 - "$rt" "$i" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/grad_place_ab_run.json"))
p = d["placement"]
print(json.dumps({"place_grad": int(sys.argv[1]), "round": int(sys.argv[2]),
                  "kernel_ms": d["kernels"]["explore"]["avg_ms"], "value": d["value"],
                  "chosen_ms": p.get("chosen_ms"), "grad_chunks": p.get("grad_chunks"), "grad_timed": p.get("grad_timed"),
                  "kept": p.get("kept"), "search_s": p.get("search_seconds", p.get("seconds")),
                  "chunks": p.get("chunks_allocated"), "tune_1x4": d["launch"]["candidates_ms"].get("1wg/cu x4")}))
PY
    tail -1 $OUT
  done
done
