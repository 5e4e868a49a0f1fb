#!/bin/bash
# SQ counter passes of tools/bench_lines.py on two corpus variants (front-end parse kernel study)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cf in 0 1; do
  PMC_BENCH="python3 tools/bench_lines.py --no-cpu --steps 1 --warmup 1 --mix 1,0,0 --compress-frac $cf" \
  PMC_OUT=gpurun_out/lpmc_cf$cf bash tools/pmc.sh sq1 sq2 tcp > gpurun_out/lpmc_cf$cf.log 2>&1 || { tail -20 gpurun_out/lpmc_cf$cf.log; exit 1; }
  echo "=== cf=$cf"; sed -n '/k_parse_lines/,/==/p' gpurun_out/lpmc_cf$cf.log
done
