# Same-process A/B of library builds with flat and per-tensor gradients
# alternating (tools/step_ab.py GRAD=ab): cSGHMC explore / Welford on ViT-L/32,
# SGLD + SGD on ResNet-101, Adam-SGHMC + SGD on ViT-L/32.
#   bash tools/ab_grad.sh [LIB ...]   (default: production vs every tools/bin flavor)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abg
libs="${*:-bayesdll_amd/libbdl_sgmcmc.so $(ls tools/bin/libbdl_*.so)}"
for spec in "vit_l_32 csghmc 1,4,1" "resnet101 sgld 2,1,1;1,4,1" "vit_l_32 adam 2,4,1;1,4,1"; do
  set -- $spec
  BACKBONE=$1 METHOD=$2 GRAD=ab ROUNDS=${ROUNDS:-3} GEOMS="$3" timeout -k 10 300 \
    python tools/step_ab.py $libs > gpurun_out/abg/ab_$1_$2.jsonl 2> gpurun_out/abg/ab_$1_$2.err || exit $?
  echo "== $1 $2"; grep summary gpurun_out/abg/ab_$1_$2.jsonl
done
