#!/bin/bash
# rocprofv3 evidence for the bench's kernels: kernel-trace stats, then the two
# HBM counters in separate passes (FETCH_SIZE and WRITE_SIZE do not fit in one
# pass on gfx950).  Output under gpurun_out/prof_${TAG}/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# --no-methods: the other methods' lines (other backbones) stay out of the
# per-kind PMC means; profile them with BENCH_ARGS="--method sgld --backbone resnet101"
BENCH="bench.py --steps ${PSTEPS:-200} --warmup 20 --no-cpu-baseline --e2e-steps 0 --no-methods ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace.log; exit 1; }
tail -3 $OUT/trace.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 24 --warmup 6 --no-cpu-baseline --e2e-steps 0 --no-methods ${BENCH_ARGS:-} > $OUT/fetch.log 2>&1 || { echo "fetch failed rc=$?"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 24 --warmup 6 --no-cpu-baseline --e2e-steps 0 --no-methods ${BENCH_ARGS:-} > $OUT/write.log 2>&1 || { echo "write failed rc=$?"; tail -20 $OUT/write.log; exit 1; }
find $OUT -name "*.csv" | head -20
