#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_x3}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 280 --timeout-method thread > "$O/tests.txt" 2>&1 \
  || { tail -40 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
bash tools/gpu_r03_xprof.sh "${1:-r03_x3}_prof"
for r in 1 2; do
  timeout -k 10 180 python bench.py --exchange --no-cpu > "$O/bench_exchange_$r.log" 2>&1 || { tail -30 "$O/bench_exchange_$r.log"; exit 1; }
  tail -1 "$O/bench_exchange_$r.log" | cut -c1-200
done
