# A/B of library builds on the noise-bearing sweeps (tools/step_ab.py), same process per case:
#   bash tools/pk_ab.sh LIB [LIB ...]     (default: the production build vs tools/bin/libbdl_*.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r4
libs="${*:-bayesdll_amd/libbdl_sgmcmc.so $(ls tools/bin/libbdl_*.so)}"
for spec in "resnet101 sgld 2,1,1;2,4,1;1,4,1" "vit_l_32 sgld 2,4,1;1,4,1;2,1,1" \
            "vit_l_32 draw 1,4,0;2,4,0" "vit_l_32 csghmc 1,4,1;1,1,1" "vit_l_32 adam 1,1,1;2,1,1;1,4,1"; do
  set -- $spec
  BACKBONE=$1 METHOD=$2 ROUNDS=3 GEOMS="$3" timeout -k 10 300 python tools/step_ab.py $libs \
    > gpurun_out/r4/pk_$1_$2.jsonl 2> gpurun_out/r4/pk_$1_$2.err || exit $?
  echo "== $1 $2"; grep summary gpurun_out/r4/pk_$1_$2.jsonl
done
