# A/B kernel timing of library variants (tools/build_variant.py); each run time-limited, stop on failure
set -o pipefail
export TMPDIR=/tmp
V="$@"
for r in 1 2; do
  for v in $V; do
    SDX_LIB=pysignalduino_amd/_lib/variants/libsdx_$v.so timeout -k 10 120 python3 tools/time_mu.py 333333 7 >> gpurun_out/ab.log 2>&1 || exit 1
  done
done
