#!/bin/bash
# Round 3: wire-format exchange + bench self-launch.  dist GPU tests (kernel vs numpy wire form,
# RCCL world 1, gloo world 2 on real kernels, bench --gpus 2 self-launch), then the default bench
# and the world-1 RCCL exchange bench (two runs each), then rocprofv3 kernel stats of --exchange.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/r03_exch
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 280 --timeout-method thread > "$O/tests.txt" 2>&1 \
  || { tail -40 "$O/tests.txt"; exit 1; }
tail -3 "$O/tests.txt"
for r in 1 2; do
  timeout -k 10 180 python bench.py --no-cpu > "$O/bench_$r.log" 2>&1 || { tail -30 "$O/bench_$r.log"; exit 1; }
  tail -1 "$O/bench_$r.log" | cut -c1-300
  timeout -k 10 180 python bench.py --exchange --no-cpu > "$O/bench_exchange_$r.log" 2>&1 || { tail -30 "$O/bench_exchange_$r.log"; exit 1; }
  tail -1 "$O/bench_exchange_$r.log" | cut -c1-300
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/ktrace" -o exch --output-format csv -- \
  python3 bench.py --exchange --no-cpu > "$O/ktrace.log" 2>&1 || { tail -30 "$O/ktrace.log"; exit 1; }
echo done
