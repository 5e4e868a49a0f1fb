#!/bin/bash
# Evidence for profiles/<round>/: PMC passes (SQ mix + FETCH/WRITE traffic), a kernel-trace
# --stats summary of the default bench command, and the default bench line (with cpu_baseline).
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 tools/pmc.sh > gpurun_out/pmc_summary.txt 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_summary.txt; exit 1; }
echo "pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats -o ks --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/kstats.log 2>&1 || { echo "kstats failed"; tail -20 gpurun_out/kstats.log; exit 1; }
echo "kstats ok"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
