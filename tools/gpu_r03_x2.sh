#!/bin/bash
# exchange kernels standalone + dist GPU tests, then the staging A/B (tools/gpu_r03_ab.sh)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_x2}
mkdir -p "$O"
timeout -k 10 120 python tools/time_exchange.py > "$O/time_exchange.log" 2>&1 || { tail -20 "$O/time_exchange.log"; exit 1; }
grep -v amdgpu.ids "$O/time_exchange.log"
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 280 --timeout-method thread > "$O/tests.txt" 2>&1 \
  || { tail -40 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
bash tools/gpu_r03_ab.sh "${1:-r03_x2}_ab" ballot
