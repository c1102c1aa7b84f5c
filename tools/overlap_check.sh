# The graph-mode update/backward overlap test on its own (first replay of the
# captured bucket nodes), then the default bench line with the graph-overlap
# e2e leg.  Stops after a fault / abort / timeout of the first step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_graph_overlap.py -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/overlap_test.log 2>&1
rc=$?
echo "== overlap test rc=$rc"; tail -n 30 gpurun_out/overlap_test.log
case $rc in 0|1) ;; *) echo "FATAL (rc=$rc): stopping"; exit $rc;; esac
BDL_BENCH_GRAPH_OVERLAP=1 timeout -k 10 420 python bench.py > gpurun_out/bench.log 2>&1
rc2=$?
echo "== bench rc=$rc2"; tail -c 6000 gpurun_out/bench.log
exit $(( rc != 0 ? rc : rc2 ))
