#!/bin/bash
# GPU-box check: smoke -> gpu tests -> short bench.  Stops at the first step that
# faults, aborts, segfaults or times out (exit 124/134/137/139 or signal exits).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; *) [ "$1" -gt 128 ] && return 0; return 1;; esac; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-smoke,tests,bench}
rc_all=0
if [[ $STEPS == *smoke* ]]; then run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || rc_all=1; fi
if [[ $STEPS == *tests* ]]; then run pytest_gpu 1000 python -u -m pytest tests -m gpu -v -rfE --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} || rc_all=1; fi
if [[ $STEPS == *bench* ]]; then run bench 400 python bench.py ${BENCH_ARGS:-} || rc_all=1; fi
exit $rc_all
