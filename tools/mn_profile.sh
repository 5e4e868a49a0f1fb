#!/bin/bash
# MN (FSK) measurement on the GPU box: bench line, kernel-trace stats, PMC traffic/SQ passes.
# usage (via gpurun): tools/mn_profile.sh   -> gpurun_out/mn/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/mn
mkdir -p "$O"
timeout -k 10 300 python3 tools/bench_mn.py > "$O/bench_mn.log" 2>&1 || { tail -20 "$O/bench_mn.log"; exit 1; }
tail -1 "$O/bench_mn.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/ktrace" -o mn --output-format csv -- \
  python3 tools/bench_mn.py --no-cpu > "$O/ktrace.log" 2>&1 || { tail -20 "$O/ktrace.log"; exit 1; }
PMC_BENCH="python3 tools/bench_mn.py --steps 3 --warmup 1 --no-cpu" PMC_OUT="$O/pmc" \
  PMC_TRAFFIC="$O/pmc_traffic_mn.json" PMC_CONFIG='{"command": "python3 tools/bench_mn.py --steps 3 --warmup 1 --no-cpu", "frames": 1000000}' \
  bash tools/pmc.sh > "$O/pmc.log" 2>&1 || { tail -20 "$O/pmc.log"; exit 1; }
tail -30 "$O/pmc.log"
