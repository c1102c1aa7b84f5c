#!/bin/bash
# One box, the bench line of every method / config (kernel-only unless noted),
# under gpurun_out/methods/: config 4 (default), config 3 (ResNet-101 SGLD),
# SGLD and Adam-SGHMC on ViT-L/32 (torch's allocator, the default); the box's clocks first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/methods
timeout -k 5 30 rocm-smi --showclocks > gpurun_out/methods/clocks.txt 2>&1 || true
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/methods/$name.json 2> gpurun_out/methods/$name.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/methods/$name.json')); r=d['roofline']; mc=r.get('mix_ceiling') or {}; print('$name', d['value'], r['kernel'], d['kernels'][r['kernel']]['avg_ms'], r['frac'], 'bare', mc.get('best_ms'), 'of_ceiling', mc.get('of_ceiling'))"
}
run csghmc_vit
run sgld_rn101 --backbone resnet101 --method sgld --no-cpu-baseline --e2e-steps 0
run sgld_vit --method sgld --no-cpu-baseline --e2e-steps 0
run adam_vit --method adam_sghmc --no-cpu-baseline --e2e-steps 0
