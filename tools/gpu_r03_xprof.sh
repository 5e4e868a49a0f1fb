#!/bin/bash
# rocprofv3 kernel stats of the exchange kernels standalone (tools/time_exchange.py)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_xprof}
mkdir -p "$O"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/kt" -o x --output-format csv -- \
  python3 tools/time_exchange.py > "$O/run.log" 2>&1 || { tail -30 "$O/run.log"; exit 1; }
grep -v amdgpu.ids "$O/run.log" | tail -2
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "xw" in r["Name"] or "xu" in r["Name"]:
        print(r["Name"][:40], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
PY
