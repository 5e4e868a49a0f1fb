#!/bin/bash
# A/B of environment settings on the default bench: tools/gpu_r03_envab.sh OUT "VAR=a" "VAR=b" ... (two rounds)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  for e in "$@"; do
    tag=$(echo "$e" | tr '=/ ' '___')
    env $e timeout -k 10 180 python bench.py --no-cpu > $O/bench_${tag}_$r.log 2>&1 || { tail -20 $O/bench_${tag}_$r.log; exit 1; }
    echo "$e run $r: $(tail -1 $O/bench_${tag}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M msgs/s", round(d["ms_per_step"],4), "ms/step", {k: round(v,4) for k,v in d.get("per_kernel_ms",{}).items()})')"
  done
done
