#!/bin/bash
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE) + SQ issue counters over tools/bench_lines.py
#   tools/pmc_lines.sh OUTDIR      -> OUTDIR/pmc/..., OUTDIR/pmc_traffic_lines.json
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$1
export PMC_BENCH="python3 tools/bench_lines.py --steps 3 --warmup 1 --no-cpu"
export PMC_OUT=$O/pmc PMC_TRAFFIC=$O/pmc_traffic_lines.json
export PMC_CONFIG='{"command": "python3 tools/bench_lines.py --steps 3 --warmup 1 --no-cpu", "lines": 1000000}'
bash tools/pmc.sh fetch write sq1
