#!/bin/bash
# the grouping sort (2 launches per pass): parity + stable-sort tests, its cost beside the launches, bench x2
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/grp2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 280 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python tools/exp_group_cost.py > $O/exp.log 2>&1 || { tail -20 $O/exp.log; exit 1; }
tail -4 $O/exp.log
for r in 1 2; do
 timeout -k 10 180 python bench.py --no-cpu > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
 echo "bench $r: $(tail -1 $O/bench_$r.log | cut -c80-150)"; done
