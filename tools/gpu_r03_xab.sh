#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_xab}
mkdir -p "$O"
shift
for v in tree "$@"; do
  if [ "$v" = tree ]; then L=pysignalduino_amd/_lib/libsdx.so; else L=pysignalduino_amd/_lib/variants/libsdx_$v.so; fi
  SDX_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/kt_$v" -o x --output-format csv -- \
    python3 tools/time_exchange.py > "$O/run_$v.log" 2>&1 || { tail -30 "$O/run_$v.log"; exit 1; }
  python3 - "$O/kt_$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "xw" in r["Name"]:
        print(sys.argv[2], r["Name"][:24], r["Calls"], r["AverageNs"])
PY
done
