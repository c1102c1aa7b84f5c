# Same-process A/B of Adam-SGHMC builds (tools/step_ab.py METHOD=adam), flat and per-tensor
# gradients: bash tools/ab_adam.sh LIB [LIB ...]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_adam
for grad in flat tensor; do
  BACKBONE=vit_l_32 METHOD=adam GRAD=$grad ROUNDS=${ROUNDS:-3} GEOMS="${GEOMS:-1,4,1;2,4,1;4,4,1;3,4,1;2,2,1}" \
    timeout -k 10 400 python tools/step_ab.py "$@" > gpurun_out/ab_adam/adam_$grad.jsonl 2>&1 || exit $?
  echo "== adam $grad"; grep summary gpurun_out/ab_adam/adam_$grad.jsonl
done
