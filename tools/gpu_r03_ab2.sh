#!/bin/bash
# A/B of library variants on the default bench: tools/gpu_r03_ab2.sh OUT VARIANT... (base = in-tree build)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L=pysignalduino_amd/_lib/variants/libsdx_$v.so; fi
    SDX_LIB=$L timeout -k 10 180 python bench.py --no-cpu > $O/bench_${v}_$r.log 2>&1 || { tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo "$v run $r: $(tail -1 $O/bench_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M msgs/s", round(d["ms_per_step"],4), "ms/step", d.get("per_kernel_ms"))')"
  done
done
