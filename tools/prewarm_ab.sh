# The driver's bench command shape (--steps 20 --warmup 5) with and without
# the prewarm, alternating in fresh processes on one box: value and explore ms.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/prewarm
for i in 1 2 3; do
  for pw in 0 1.0; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --prewarm-seconds $pw --no-methods \
      --e2e-steps 0 --no-cpu-baseline --no-aux > gpurun_out/prewarm/run_${i}_${pw}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], d['value'], d['kernels']['explore']['avg_ms'], d['roofline']['frac'])" gpurun_out/prewarm/run_${i}_${pw}.json $pw
  done
done
