#!/bin/bash
# Round-6 A/B: the pipelined cSGHMC collect sweep (make flavor F=pipe
# D=-DBDL_PIPE_CSGHMC_COLLECT) against the production build, same process,
# builds alternating (tools/step_ab.py: explore, Welford collect and Welford
# init at every geometry), after the collect paths' parity tests under the
# flavor.  Usage: bash tools/ab_collect_pipe.sh PROD.so PIPE.so
set -u
cd "${GRAFT_REPO_ROOT:-.}"
PROD=$1
PIPE=$2
mkdir -p gpurun_out/ab_pipe
BDL_SGMCMC_LIB=$(readlink -f "$PIPE") timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_multi_run.py \
  tests/test_gpu_fullsize_parity.py > gpurun_out/ab_pipe/parity_flavor.log 2>&1 \
  || { tail -30 gpurun_out/ab_pipe/parity_flavor.log; exit 1; }
tail -2 gpurun_out/ab_pipe/parity_flavor.log
for spec in "flat 1,1,1;2,1,1;1,2,1;1,4,1;2,2,1" "tensor 1,1,1;2,1,1;1,4,1"; do
  set -- $spec
  BACKBONE=vit_l_32 METHOD=csghmc GRAD=$1 ROUNDS=${ROUNDS:-3} GEOMS="$2" COLLECT_ALL=1 INIT=1 \
    timeout -k 10 300 python tools/step_ab.py $PROD $PIPE > gpurun_out/ab_pipe/ab_$1.jsonl \
    2> gpurun_out/ab_pipe/ab_$1.err || exit $?
  echo "== $1"; grep summary gpurun_out/ab_pipe/ab_$1.jsonl
done
