#!/bin/bash
# k_pulses MU / MS standalone (tools/time_mu.py) for library variants, two rounds: OUT VARIANT...
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L=pysignalduino_amd/_lib/variants/libsdx_$v.so; fi
    SDX_LIB=$L timeout -k 10 120 python tools/time_mu.py > $O/time_${v}_$r.log 2>&1 || { tail -20 $O/time_${v}_$r.log; exit 1; }
    echo "$v $r: $(tail -1 $O/time_${v}_$r.log)"
  done
done
