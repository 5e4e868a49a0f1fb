#!/bin/bash
# round 3 (session 2) measurement set: whole -m gpu suite + smoke, bench (CPU baseline once, then x2
# without), --exchange, line bench, e2e pipeline, rocprofv3 kernel stats of bench.py and bench_lines,
# PMC passes (sq1 sq2 fetch write) -> gpurun_out/<out>/pmc_traffic.json
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/tests.txt 2>&1 \
  || { tail -60 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_cpu.log 2>&1 || { tail -30 $O/bench_cpu.log; exit 1; }
tail -1 $O/bench_cpu.log | cut -c1-200
for r in 1 2; do
  timeout -k 10 180 python bench.py --no-cpu > $O/bench_$r.log 2>&1 || { tail -30 $O/bench_$r.log; exit 1; }
  tail -1 $O/bench_$r.log | cut -c1-200
done
timeout -k 10 180 python bench.py --exchange --no-cpu > $O/bench_exchange.log 2>&1 || { tail -30 $O/bench_exchange.log; exit 1; }
tail -1 $O/bench_exchange.log | cut -c1-200
timeout -k 10 300 python tools/bench_lines.py --no-cpu > $O/bench_lines.log 2>&1 || { tail -30 $O/bench_lines.log; exit 1; }
tail -1 $O/bench_lines.log | cut -c1-200
timeout -k 10 400 python -u tools/bench_lines_e2e.py --check > $O/lines_e2e.log 2>&1 || { tail -30 $O/lines_e2e.log; exit 1; }
tail -1 $O/lines_e2e.log | cut -c1-300
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt_bench -o b --output-format csv -- \
  python3 bench.py --no-cpu > $O/kt_bench.log 2>&1 || { tail -30 $O/kt_bench.log; exit 1; }
tail -1 $O/kt_bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_lines -o l --output-format csv -- \
  python3 tools/bench_lines.py --no-cpu > $O/kt_lines.log 2>&1 || { tail -30 $O/kt_lines.log; exit 1; }
PMC_OUT=$O/pmc PMC_TRAFFIC=$O/pmc_traffic.json bash tools/pmc.sh sq1 sq2 fetch write > $O/pmc.log 2>&1 || { tail -30 $O/pmc.log; exit 1; }
tail -12 $O/pmc.log
echo done
