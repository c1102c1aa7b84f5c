set -u
mkdir -p gpurun_out/e2e_compare
BACKBONE=mlp_mnist BATCH=128 STEPS=200 timeout -k 10 300 python tools/e2e_compare.py > gpurun_out/e2e_compare/mlp_mnist.jsonl 2> gpurun_out/e2e_compare/mlp_mnist.err || { tail gpurun_out/e2e_compare/mlp_mnist.err; exit 1; }
cat gpurun_out/e2e_compare/mlp_mnist.jsonl
BACKBONE=vit_l_32 BATCH=16 STEPS=20 timeout -k 10 400 python tools/e2e_compare.py > gpurun_out/e2e_compare/vit_l_32.jsonl 2> gpurun_out/e2e_compare/vit_l_32.err || { tail gpurun_out/e2e_compare/vit_l_32.err; exit 1; }
cat gpurun_out/e2e_compare/vit_l_32.jsonl
BACKBONE=resnet101 BATCH=16 STEPS=20 timeout -k 10 400 python tools/e2e_compare.py > gpurun_out/e2e_compare/resnet101.jsonl 2> gpurun_out/e2e_compare/resnet101.err || { tail gpurun_out/e2e_compare/resnet101.err; exit 1; }
cat gpurun_out/e2e_compare/resnet101.jsonl
