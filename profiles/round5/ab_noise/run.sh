# Same-process A/B of library builds over the Philox-bearing step sweeps (tools/step_ab.py):
# ResNet-101 SGLD (+ its collect) and the ViT-L/32 cSGHMC Welford collect.
#   bash tools/ab_noise.sh LIB [LIB ...]
set -u
LIBS="$*"
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab_noise
for spec in "resnet101 sgld flat 2,1,1;1,4,1;1,1,1;3,1,1" "resnet101 sgld tensor 2,1,1;1,4,1" \
            "vit_l_32 csghmc flat 1,1,1;1,4,1" "vit_l_32 csghmc flat 1,4,1;2,1,1"; do
  set -- $spec
  tag=$1_$2_$3_${4%%;*}
  BACKBONE=$1 METHOD=$2 GRAD=$3 ROUNDS=${ROUNDS:-3} GEOMS="$4" timeout -k 10 300 \
    python tools/step_ab.py $LIBS > gpurun_out/ab_noise/$tag.jsonl 2>&1 || exit $?
  echo "== $tag"; grep summary gpurun_out/ab_noise/$tag.jsonl
done
