#!/bin/bash
# Round 3: the whole -m gpu suite, then bench default + --exchange (two runs each), rocprofv3
# kernel stats of --exchange.  Usage: tools/gpu_r03_all.sh <outdir-name>
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_all}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > "$O/tests.txt" 2>&1 \
  || { tail -60 "$O/tests.txt"; exit 1; }
tail -3 "$O/tests.txt"
for r in 1 2; do
  timeout -k 10 180 python bench.py --no-cpu > "$O/bench_$r.log" 2>&1 || { tail -30 "$O/bench_$r.log"; exit 1; }
  tail -1 "$O/bench_$r.log" | cut -c1-250
  timeout -k 10 180 python bench.py --exchange --no-cpu > "$O/bench_exchange_$r.log" 2>&1 || { tail -30 "$O/bench_exchange_$r.log"; exit 1; }
  tail -1 "$O/bench_exchange_$r.log" | cut -c1-250
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/ktrace" -o exch --output-format csv -- \
  python3 bench.py --exchange --no-cpu > "$O/ktrace.log" 2>&1 || { tail -30 "$O/ktrace.log"; exit 1; }
echo done
