set -u
mkdir -p gpurun_out/ab_sghmc
for spec in "resnet101 flat 2,1,1;1,4,1;1,1,1" "vit_l_32 tensor 2,1,1;1,4,1"; do
  set -- $spec
  tag=$1_$2
  BACKBONE=$1 METHOD=sghmc GRAD=$2 ROUNDS=3 GEOMS="$3" timeout -k 10 300 \
    python tools/step_ab.py tools/bin/libbdl_base.so tools/bin/libbdl_pc.so tools/bin/libbdl_pcgg.so > gpurun_out/ab_sghmc/$tag.jsonl 2>&1 || exit $?
  echo "== $tag"; grep summary gpurun_out/ab_sghmc/$tag.jsonl
done
