#!/bin/bash
# k_parse_lines at 6 waves/SIMD (80 VGPRs) vs 5 (libsdx_pl5.so = the build before): front-end
# parity tests on the new build, then tools/bench_lines.py twice per library.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/pl6
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_lines.py tests/test_json.py tests/test_controller.py -m gpu -x -v --timeout 150 \
  --timeout-method thread > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
for r in 1 2; do
  for lib in pysignalduino_amd/_lib/variants/libsdx_pl5.so pysignalduino_amd/_lib/libsdx.so; do
    SDX_LIB=$lib timeout -k 10 200 python tools/bench_lines.py --no-cpu > "$O/lines_$(basename $lib .so)_$r.log" 2>&1 \
      || { tail -30 "$O/lines_$(basename $lib .so)_$r.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/lines_$(basename $lib .so)_$r.log').read().strip().splitlines()[-1]); print('$lib', round(d['value']/1e6,1), {k: round(v,3) for k,v in d['per_kernel_ms'].items()})"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/ktrace" -o lines --output-format csv -- \
  python3 tools/bench_lines.py --no-cpu > "$O/ktrace.log" 2>&1 || { tail -30 "$O/ktrace.log"; exit 1; }
echo done
