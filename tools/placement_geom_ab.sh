mkdir -p gpurun_out
for i in 1 2 3; do
  for b in 1 2; do
    BDL_PLACEMENT_BPC=$b timeout -k 10 200 python3 bench.py --method sgld --no-cpu-baseline --e2e-steps 0 --no-aux > gpurun_out/pg_vit_${b}_$i.json 2>/dev/null || exit 1
    BDL_PLACEMENT_BPC=$b timeout -k 10 200 python3 bench.py --method sgld --backbone resnet101 --no-cpu-baseline --e2e-steps 0 --no-aux > gpurun_out/pg_rn_${b}_$i.json 2>/dev/null || exit 1
    echo "$i $b done"
  done
done
