#!/bin/bash
# Round-4 GPU box: smoke -> full pytest -m gpu -> default bench (gpu_check.sh),
# then every method's bench line (method_benches.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh || exit $?
bash tools/method_benches.sh
