#!/bin/bash
# last check of the session: the whole -m gpu suite at HEAD, then the MU cost-table and index-prefetch A/Bs
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/r03_last; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/tests.txt 2>&1 \
  || { tail -60 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/gpu_r03_envab.sh mucost SDX_MU_COSTS=r2 SDX_MU_COSTS=r3 && bash tools/gpu_r03_timeab.sh pf pf
