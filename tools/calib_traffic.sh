#!/bin/bash
# Counter calibration: tools/_bin/calib_traffic (built on the CPU side:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/calib_traffic.hip -o tools/_bin/calib_traffic)
# under one rocprofv3 --pmc pass per counter, then the ratios.  Usage: tools/calib_traffic.sh OUT
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/calib}
mkdir -p "$O"
timeout -k 10 120 ./tools/_bin/calib_traffic > "$O/known.txt" 2>&1 || { echo "calib run failed"; cat "$O/known.txt"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$O/$c" -o "$c" --output-format csv -- ./tools/_bin/calib_traffic > "$O/$c.log" 2>&1 \
    || { echo "pmc $c failed"; tail -20 "$O/$c.log"; exit 1; }
done
python3 tools/calib_traffic.py "$O"
