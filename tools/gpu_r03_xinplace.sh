#!/bin/bash
# in-place exchange (sdx_exchange_pack_into): dist GPU tests, bench --exchange x2 vs default, MU finish sub-phases
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/xinplace; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for f in "" "--exchange"; do
    timeout -k 10 180 python bench.py --no-cpu $f > $O/bench${f}_$r.log 2>&1 || { tail -30 $O/bench${f}_$r.log; exit 1; }
    echo "$f $r: $(tail -1 $O/bench${f}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M msgs/s", round(d["ms_per_step"],4), "ms/step", d.get("per_kernel_ms"))')"
  done
done
SDX_LIB=pysignalduino_amd/_lib/variants/libsdx_prof.so timeout -k 10 300 python tools/prof_phases.py > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
head -28 $O/phases.log
