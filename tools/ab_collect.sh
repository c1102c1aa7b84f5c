# Same-process A/B of library builds on the ViT-L/32 cSGHMC Welford collect (collect kind at
# the first geometry of each spec), flat and per-tensor gradients:
#   bash tools/ab_collect.sh LIB [LIB ...]
set -u
LIBS="$*"
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_collect
for spec in "flat 1,1,1" "flat 1,4,1" "tensor 1,1,1" "flat 2,4,1"; do
  set -- $spec
  tag=$1_$2
  BACKBONE=vit_l_32 METHOD=csghmc GRAD=$1 ROUNDS=${ROUNDS:-3} GEOMS="$2" timeout -k 10 300 \
    python tools/step_ab.py $LIBS > gpurun_out/ab_collect/$tag.jsonl 2>&1 || exit $?
  echo "== $tag"; grep summary gpurun_out/ab_collect/$tag.jsonl
done
