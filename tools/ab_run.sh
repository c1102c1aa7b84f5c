# Same-process A/B of library builds (tools/step_ab.py) over the explore /
# Welford (flat and per-tensor gradients) and ResNet-101 SGLD sweeps:
#   make -C bayesdll_amd/csrc flavor F=name D="-D..."   (builds tools/bin/libbdl_name.so)
#   bash tools/ab_run.sh [LIB ...]     (default: production vs every tools/bin flavor)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
libs="${*:-bayesdll_amd/libbdl_sgmcmc.so $(ls tools/bin/libbdl_*.so)}"
for spec in "vit_l_32 csghmc flat 1,4,1;1,1,1;2,1,1" "vit_l_32 csghmc tensor 1,4,1;1,1,1;2,1,1" \
            "resnet101 sgld flat 2,1,1;1,4,1;1,1,1"; do
  set -- $spec
  BACKBONE=$1 METHOD=$2 GRAD=$3 ROUNDS=${ROUNDS:-3} GEOMS="$4" timeout -k 10 300 \
    python tools/step_ab.py $libs > gpurun_out/ab/ab_$1_$2_$3.jsonl 2> gpurun_out/ab/ab_$1_$2_$3.err || exit $?
  echo "== $1 $2 $3"; grep summary gpurun_out/ab/ab_$1_$2_$3.jsonl
done
