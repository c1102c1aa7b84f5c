set -u
mkdir -p gpurun_out/ab_ord
libs="tools/bin/libbdl_base.so tools/bin/libbdl_ord.so"
for spec in "resnet101 sgld flat 1,1,1;2,1,1;1,4,1" "vit_l_32 csghmc flat 1,1,1;1,4,1;2,1,1" "vit_l_32 csghmc tensor 1,1,1;1,4,1" "resnet101 sgld flat 2,1,1;1,1,1"; do
  set -- $spec
  BACKBONE=$1 METHOD=$2 GRAD=$3 ROUNDS=3 GEOMS="$4" timeout -k 10 300 \
    python tools/step_ab.py $libs > gpurun_out/ab_ord/ab_$1_$2_$3_${4%%;*}.jsonl 2>&1 || exit $?
  echo "== $1 $2 $3 $4"; grep summary gpurun_out/ab_ord/ab_$1_$2_$3_${4%%;*}.jsonl
done
