#!/bin/bash
# A/B of the placement search's second timing round (BDL_PLACEMENT_RETIME=0 vs
# ${RETIME:-3}), alternating fresh bench processes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/retime_ab.jsonl
: > $OUT
for i in $(seq 1 ${ROUNDS:-6}); do
  for rt in 0 ${RETIME:-3}; do
    BDL_PLACEMENT_RETIME=$rt timeout -k 10 200 python bench.py --no-aux --no-cpu-baseline \
      --e2e-steps 0 > gpurun_out/retime_ab_run.json 2> gpurun_out/retime_ab_run.err || exit 1
    python3 - "$rt" "$i" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/retime_ab_run.json"))
p = d["placement"]
print(json.dumps({"retime": int(sys.argv[1]), "round": int(sys.argv[2]),
                  "kernel_ms": d["kernels"]["explore"]["avg_ms"], "value": d["value"],
                  "chosen_ms": p.get("chosen_ms"), "retimed_ms": p.get("retimed_ms"),
                  "kept": p.get("kept"), "search_s": p.get("search_seconds", p.get("seconds")),
                  "chunks": p.get("chunks_allocated"), "tune_1x4": d["launch"]["candidates_ms"].get("1wg/cu x4")}))
PY
    tail -1 $OUT
  done
done
