#!/bin/bash
# world-1 RCCL exchange bench after the count-copy fix (two runs + rocprofv3 kernel stats), the
# RCCL exchange test, then the front-end profile (tools/lines_profile.sh).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/exch
mkdir -p "$O"
timeout -k 10 200 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 150 --timeout-method thread > "$O/tests.txt" 2>&1 \
  || { tail -30 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
for r in 1 2; do
  timeout -k 10 180 python bench.py --exchange --no-cpu > "$O/bench_exchange_$r.log" 2>&1 || { tail -30 "$O/bench_exchange_$r.log"; exit 1; }
  tail -1 "$O/bench_exchange_$r.log" | cut -c1-400
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/ktrace" -o exch --output-format csv -- \
  python3 bench.py --exchange --no-cpu > "$O/ktrace.log" 2>&1 || { tail -30 "$O/ktrace.log"; exit 1; }
bash tools/lines_profile.sh
