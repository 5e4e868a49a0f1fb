#!/bin/bash
# A/B of the MS grouping key (sdx_group.hip SDX_MS_KEY 0-3): k_pulses<MU>/<MS> time incl. grouping,
# two rounds per library, 333k messages.  Build the variants first:
#   for v in 1 2 3; do python tools/build_variant.py mskey$v --unit sdx_group.hip -DSDX_MS_KEY=$v; done
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/mskey
mkdir -p "$O"
V=pysignalduino_amd/_lib/variants
for r in 1 2; do
  for lib in pysignalduino_amd/_lib/libsdx.so $V/libsdx_mskey1.so $V/libsdx_mskey2.so $V/libsdx_mskey3.so; do
    SDX_LIB=$lib timeout -k 10 120 python tools/time_mu.py 333333 10 >> "$O/time.log" 2>&1 || { tail -20 "$O/time.log"; exit 1; }
  done
done
cat "$O/time.log"
