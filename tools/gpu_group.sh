# grouped vs plain message order: GPU test suite, kernel times of both orders, kernel breakdown
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/check.log 2>&1 || { tail -40 gpurun_out/check.log; exit 1; }
tail -2 gpurun_out/check.log
timeout -k 10 120 python3 tools/time_mu.py 333333 7 || exit 1
SDX_NOGROUP=1 timeout -k 10 120 python3 tools/time_mu.py 333333 7 || exit 1
rm -rf gpurun_out/gprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o gp --output-format csv -- python3 tools/time_mu.py 333333 5 > gpurun_out/gprof.log 2>&1 || exit 1
