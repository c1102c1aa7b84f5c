#!/bin/bash
# N fresh default bench processes (kernel-only), the whole placement info of
# each under gpurun_out/placement_info.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/placement_info.jsonl
: > $OUT
for i in $(seq 1 ${RUNS:-6}); do
  timeout -k 10 200 python bench.py --no-aux --no-cpu-baseline --e2e-steps 0 \
    > gpurun_out/pi_run.json 2> gpurun_out/pi_run.err || exit 1
  python3 - "$i" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/pi_run.json"))
print(json.dumps({"run": int(sys.argv[1]), "kernel_ms": d["kernels"]["explore"]["avg_ms"],
                  "value": d["value"], "placement": d["placement"],
                  "tune": d["launch"].get("candidates_ms")}))
PY
  python3 -c "import json; d=[json.loads(l) for l in open('$OUT')][-1]; p=d['placement']; print(d['run'], d['kernel_ms'], p['chosen_ms'], p['kept'], p['chunks_allocated'], p['pair_ms_min'], p['pair_ms_median'])"
done
