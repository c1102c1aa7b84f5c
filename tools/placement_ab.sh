#!/bin/bash
# A/B of the allocators on one box: torch's (BDL_PLACEMENT=0), physical chunks
# in allocation order (order), chunks with pair search (search); alternating
# full bench runs (kernel-only), one JSON line each under gpurun_out/ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in ${ROUNDS:-1 2}; do
  for m in 0 order search; do
    BDL_PLACEMENT=$m timeout -k 10 200 python bench.py --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS:-} \
      > gpurun_out/ab/$m.$r.json 2> gpurun_out/ab/$m.$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$m.$r.json')); k=d['kernels']; print('$m', $r, d['value'], k['explore']['avg_ms'], d.get('aux_kernels'), d.get('placement'))"
  done
done
