#!/bin/bash
# Round-4 GPU box: the kernel / geometry / Adam / draw tests, then every
# method's bench line (tools/method_benches.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpu_geometry.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -v -rfE --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4/pytest_kernels.log
[ $rc -ne 0 ] && exit $rc
bash tools/method_benches.sh
