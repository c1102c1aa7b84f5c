#!/bin/bash
# A/B of the placement search's pair timing: all ordered chunk pairs vs every
# chunk against chunk 0 ("ref"), alternating fresh bench processes on one box.
# One JSON summary line per run under gpurun_out/pairs_ab.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/pairs_ab.jsonl
: > $OUT
for i in $(seq 1 ${ROUNDS:-3}); do
  for mode in all ref; do
    for method in ${METHODS:-csghmc}; do
      BDL_PLACEMENT_PAIRS=$mode timeout -k 10 200 python bench.py --method $method --no-aux \
        --no-cpu-baseline --e2e-steps 0 > gpurun_out/pairs_ab_run.json 2> gpurun_out/pairs_ab_run.err || exit 1
      python3 - "$mode" "$method" "$i" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/pairs_ab_run.json"))
p = d["placement"]
k = d["roofline"]["kernel"]
print(json.dumps({"mode": sys.argv[1], "method": sys.argv[2], "round": int(sys.argv[3]),
                  "kernel_ms": d["kernels"][k]["avg_ms"], "value": d["value"],
                  "chosen_ms": p.get("chosen_ms"), "kept": p.get("kept"),
                  "search_s": p.get("search_seconds", p.get("seconds")),
                  "pairs_timed": p.get("pairs_timed"), "chunks": p.get("chunks_allocated"),
                  "rounds": p.get("escalation_rounds"),
                  "composites_ms": p.get("composites_ms"), "torch_ms": p.get("torch_ms")}))
PY
      tail -1 $OUT
    done
  done
done
