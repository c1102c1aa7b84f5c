#!/bin/bash
# Placement GPU tests, then N default bench processes (kernel-only) with their
# placement summaries, under gpurun_out/placement_check.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_draw_placement.py \
  -q -x -k "placed or placement or place_one or draw" --timeout 200 --timeout-method thread \
  > gpurun_out/placement_tests.log 2>&1 || { tail -30 gpurun_out/placement_tests.log; exit 1; }
tail -2 gpurun_out/placement_tests.log
OUT=gpurun_out/placement_check.jsonl
: > $OUT
for i in $(seq 1 ${RUNS:-4}); do
  for method in ${METHODS:-csghmc}; do
    timeout -k 10 200 python bench.py --method $method --no-aux --no-cpu-baseline --e2e-steps 0 \
      > gpurun_out/pc_run.json 2> gpurun_out/pc_run.err || exit 1
    python3 - "$method" "$i" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/pc_run.json"))
p = d["placement"]
k = d["roofline"]["kernel"]
print(json.dumps({"method": sys.argv[1], "run": int(sys.argv[2]), "kernel_ms": d["kernels"][k]["avg_ms"],
                  "value": d["value"], "chosen_ms": p.get("chosen_ms"), "kept": p.get("kept"),
                  "search_s": p.get("search_seconds", p.get("seconds")), "chunks": p.get("chunks_allocated"),
                  "rounds": p.get("escalation_rounds"), "pairs_timed": p.get("pairs_timed"),
                  "pair_ms_min": p.get("pair_ms_min"), "pair_ms_median": p.get("pair_ms_median"),
                  "ref_ms": p.get("ref_ms"), "composites_ms": p.get("composites_ms"),
                  "torch_ms": p.get("torch_ms")}))
PY
    tail -1 $OUT | cut -c1-220
  done
done
