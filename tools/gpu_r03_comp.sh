#!/bin/bash
# Round 3: k_parse_comp from LDS -- front-end GPU tests, A/B of the parse (tree vs the
# global-memory variant), and the phase profile of the tree's kernel (SDX_LPROF build).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/r03_comp
mkdir -p "$O"
V=pysignalduino_amd/_lib/variants
timeout -k 10 400 python -u -m pytest tests/test_lines.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for r in 1 2; do
  for v in tree scanw1 scanw8; do
    if [ "$v" = tree ]; then L=pysignalduino_amd/_lib/libsdx.so; else L=$V/libsdx_$v.so; fi
    SDX_LIB=$L timeout -k 10 300 python tools/bench_lines.py --no-cpu > "$O/bench_${v}_$r.log" 2>&1 || { tail -20 "$O/bench_${v}_$r.log"; exit 1; }
    echo "$v $(tail -1 "$O/bench_${v}_$r.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M lines/s", d.get("per_kernel_ms"))')"
  done
done
if [ -f $V/libsdx_lprof.so ]; then
  SDX_LIB=$V/libsdx_lprof.so timeout -k 10 300 python -u tools/prof_lines.py > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
  grep -v amdgpu.ids "$O/prof.log"
fi
if [ -f $V/libsdx_lprofg.so ]; then
  SDX_LIB=$V/libsdx_lprofg.so timeout -k 10 300 python -u tools/prof_lines.py > "$O/prof_global.log" 2>&1 || { tail -20 "$O/prof_global.log"; exit 1; }
  grep -v amdgpu.ids "$O/prof_global.log"
fi
