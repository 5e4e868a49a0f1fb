#!/bin/bash
# general path tests + timing, the e2e line pipeline, exchange kernels + dist tests, staging A/B
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_batch}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_general.py tests/test_lines.py -m gpu -x -v --timeout 280 --timeout-method thread > "$O/tests_general.txt" 2>&1 \
  || { tail -40 "$O/tests_general.txt"; exit 1; }
tail -2 "$O/tests_general.txt"
timeout -k 10 240 python tools/time_general.py --cpu 310 > "$O/time_general.log" 2>&1 || { tail -20 "$O/time_general.log"; exit 1; }
grep -v amdgpu.ids "$O/time_general.log"
timeout -k 10 300 python tools/bench_lines_e2e.py --check > "$O/lines_e2e.log" 2>&1 || { tail -20 "$O/lines_e2e.log"; exit 1; }
tail -1 "$O/lines_e2e.log" | cut -c1-900
bash tools/gpu_r03_x2.sh "${1:-r03_batch}_x2"
