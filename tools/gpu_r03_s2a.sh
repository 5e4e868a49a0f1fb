#!/bin/bash
# round 3 session 2: whole -m gpu suite, MC long-launch A/B, controller bench (objects / json)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_s2a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/tests.txt 2>&1 \
  || { tail -60 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for pub in objects json; do
  timeout -k 10 300 python tools/bench_controller.py --publish $pub > $O/controller_$pub.log 2>&1 || { tail -20 $O/controller_$pub.log; exit 1; }
  tail -1 $O/controller_$pub.log | cut -c1-300
done
bash tools/gpu_r03_ab2.sh ${1:-r03_s2a}/ab nomclong
