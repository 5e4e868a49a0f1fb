#!/bin/bash
# Round 3: SWAR staging A/B (k_pulses MU/MS kernel times, ballot variant vs tree), parity on the
# tree build, then tools/gpu_r03_all.sh (whole suite, benches, exchange profile).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_stage}
mkdir -p "$O"
V=pysignalduino_amd/_lib/variants
for r in 1 2; do
  SDX_LIB=$V/libsdx_ballot.so timeout -k 10 120 python tools/time_mu.py >> "$O/ab.log" 2>&1 || { tail -20 "$O/ab.log"; exit 1; }
  timeout -k 10 120 python tools/time_mu.py >> "$O/ab.log" 2>&1 || { tail -20 "$O/ab.log"; exit 1; }
done
grep -v amdgpu.ids "$O/ab.log"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -v --timeout 280 --timeout-method thread > "$O/parity.txt" 2>&1 \
  || { tail -40 "$O/parity.txt"; exit 1; }
tail -2 "$O/parity.txt"
bash tools/gpu_r03_all.sh "${1:-r03_stage}_all"
