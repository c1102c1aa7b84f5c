#!/bin/bash
# Round-4 GPU box check: the pipelined-Adam A/B (one process, alternating
# builds), then smoke -> full pytest -m gpu -> default bench (tools/gpu_check.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
if [ -n "${AB:-1}" ] && [ "${AB:-1}" != 0 ]; then
  METHOD=adam ROUNDS=3 GEOMS="1,1,1;1,2,1;2,1,1;2,2,1;1,4,1;4,4,1" timeout -k 10 500 \
    python tools/step_ab.py bayesdll_amd/libbdl_sgmcmc.so tools/bin/libbdl_adampipe.so \
    > gpurun_out/r4/adam_pipe_ab.jsonl 2> gpurun_out/r4/adam_pipe_ab.err
  rc=$?; echo "ab_rc=$rc"; grep summary gpurun_out/r4/adam_pipe_ab.jsonl
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
bash tools/gpu_check.sh
