#!/bin/bash
# Round 3 A/B: time_mu (k_pulses MU/MS incl. grouping) and the default bench for the tree build and
# the listed variants (pysignalduino_amd/_lib/variants/libsdx_<name>.so), alternating, two rounds.
# usage: tools/gpu_r03_ab.sh OUTDIR name1 [name2 ...]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/$1
shift
mkdir -p "$O"
V=pysignalduino_amd/_lib/variants
for r in 1 2; do
  for v in tree "$@"; do
    if [ "$v" = tree ]; then L=pysignalduino_amd/_lib/libsdx.so; else L=$V/libsdx_$v.so; fi
    SDX_LIB=$L timeout -k 10 120 python tools/time_mu.py >> "$O/time_mu.log" 2>&1 || { tail -20 "$O/time_mu.log"; exit 1; }
    SDX_LIB=$L timeout -k 10 180 python bench.py --no-cpu > "$O/bench_${v}_$r.log" 2>&1 || { tail -20 "$O/bench_${v}_$r.log"; exit 1; }
    python - "$O/bench_${v}_$r.log" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"] / 1e6, 1), "M msgs/s", {k: round(v, 3) for k, v in d["per_kernel_ms"].items()},
      "group", round(d["group_ms"], 3))
PY
  done
done
grep -v amdgpu.ids "$O/time_mu.log"
