set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in base ilp memclause base; do
  SDX_LIB=pysignalduino_amd/_lib/variants/libsdx_$v.so timeout -k 10 120 python tools/time_mu.py 333333 7 > gpurun_out/v_$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/v_$v.log)"
done
