set -u
mkdir -p gpurun_out/ab_g
for spec in "resnet101 sgld flat 2,1,1;1,4,1" "resnet101 sgld tensor 2,1,1;3,1,1" "vit_l_32 sgld tensor 1,4,1;2,1,1"; do
  set -- $spec
  tag=$1_$2_$3_${4%%;*}
  BACKBONE=$1 METHOD=$2 GRAD=$3 ROUNDS=3 GEOMS="$4" timeout -k 10 300 \
    python tools/step_ab.py tools/bin/libbdl_base.so tools/bin/libbdl_g.so tools/bin/libbdl_sbg.so > gpurun_out/ab_g/$tag.jsonl 2>&1 || exit $?
  echo "== $tag"; grep summary gpurun_out/ab_g/$tag.jsonl
done
