#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_lpt}
mkdir -p "$O"
for r in 1 2 3; do
  timeout -k 10 120 python tools/time_mu.py >> "$O/time_mu.log" 2>&1 || { tail -20 "$O/time_mu.log"; exit 1; }
  SDX_MU_ORDER=size timeout -k 10 120 python tools/time_mu.py >> "$O/time_mu.log" 2>&1 || { tail -20 "$O/time_mu.log"; exit 1; }
done
grep -v amdgpu.ids "$O/time_mu.log"
for r in 1 2; do
  timeout -k 10 180 python bench.py --no-cpu > "$O/bench_$r.log" 2>&1 || { tail -30 "$O/bench_$r.log"; exit 1; }
  tail -1 "$O/bench_$r.log" | cut -c1-120
done
