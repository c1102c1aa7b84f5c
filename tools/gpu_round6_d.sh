set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/ab_spills.sh tools/bin/libbdl_head.so bayesdll_amd/libbdl_sgmcmc.so > gpurun_out/ab_spills.txt 2>&1 || { tail gpurun_out/ab_spills.txt; exit 1; }
bash tools/ab_collect_pipe.sh bayesdll_amd/libbdl_sgmcmc.so tools/bin/libbdl_pipe.so > gpurun_out/ab_pipe.txt 2>&1 || { tail -30 gpurun_out/ab_pipe.txt; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
echo done
