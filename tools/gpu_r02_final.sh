#!/bin/bash
# End-of-round-2 check on the GPU box: the whole -m gpu suite, smoke(), the default bench line,
# the world-1 RCCL exchange bench (--exchange) and the rocprofv3 kernel stats of the default bench.
# usage (via gpurun): bash tools/gpu_r02_final.sh   -> gpurun_out/final/...
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/final
mkdir -p "$O"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$O/gpu_tests.txt" 2>&1 \
  || { tail -30 "$O/gpu_tests.txt"; exit 1; }
tail -1 "$O/gpu_tests.txt"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$O/smoke.txt" 2>&1 \
  || { tail -30 "$O/smoke.txt"; exit 1; }
tail -1 "$O/smoke.txt"
timeout -k 10 180 python bench.py > "$O/bench_default.log" 2>&1 || { tail -30 "$O/bench_default.log"; exit 1; }
tail -1 "$O/bench_default.log"
timeout -k 10 180 python bench.py --exchange --no-cpu > "$O/bench_exchange_rccl_w1.log" 2>&1 \
  || { tail -30 "$O/bench_exchange_rccl_w1.log"; exit 1; }
tail -1 "$O/bench_exchange_rccl_w1.log"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/ktrace" -o bench --output-format csv -- \
  python3 bench.py --no-cpu > "$O/ktrace.log" 2>&1 || { tail -30 "$O/ktrace.log"; exit 1; }
echo done
