#!/bin/bash
# round-3 measurement set: e2e line pipeline (two runs + 500k chunks), the default bench's rocprofv3
# kernel stats, and the PMC passes (sq1 sq2 fetch write) -> gpurun_out/pmc_traffic_r03.json
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/r03_meas
mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 300 python tools/bench_lines_e2e.py --check > "$O/e2e_$r.log" 2>&1 || { tail -20 "$O/e2e_$r.log"; exit 1; }
  tail -1 "$O/e2e_$r.log" | cut -c200-700
done
timeout -k 10 300 python tools/bench_lines_e2e.py --chunk 500000 --passes 4 > "$O/e2e_500k.log" 2>&1 || { tail -20 "$O/e2e_500k.log"; exit 1; }
tail -1 "$O/e2e_500k.log" | cut -c200-700
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/kt" -o bench --output-format csv -- \
  python3 bench.py --no-cpu > "$O/bench_prof.log" 2>&1 || { tail -30 "$O/bench_prof.log"; exit 1; }
tail -1 "$O/bench_prof.log" | cut -c1-200
PMC_OUT=$O/pmc PMC_TRAFFIC=gpurun_out/pmc_traffic_r03.json bash tools/pmc.sh sq1 sq2 fetch write > "$O/pmc.log" 2>&1 || { tail -30 "$O/pmc.log"; exit 1; }
tail -25 "$O/pmc.log"
