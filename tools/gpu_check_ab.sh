# correctness of the in-tree library (the MU/MS parity tests), then A/B timing of variants
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_units.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/check.log 2>&1 || { tail -30 gpurun_out/check.log; exit 1; }
tail -2 gpurun_out/check.log
bash tools/gpu_ab.sh "$@"
