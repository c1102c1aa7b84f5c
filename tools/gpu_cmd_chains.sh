set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chains.py > gpurun_out/chains.txt 2>&1; rc=$?
tail -30 gpurun_out/chains.txt
case $rc in 124|134|137|139) exit $rc;; esac
PROBE=all timeout -k 10 300 ./tools/hbm_probe > gpurun_out/hbm_probe_all.txt 2>&1
echo "probe rc=$?"
exit $rc
