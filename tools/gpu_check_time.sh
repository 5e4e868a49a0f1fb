# correctness of the in-tree library (the whole -m gpu suite), then the in-tree MU/MS kernel times
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/check.log 2>&1 || { tail -40 gpurun_out/check.log; exit 1; }
tail -2 gpurun_out/check.log
for r in 1 2; do timeout -k 10 120 python3 tools/time_mu.py 333333 7 || exit 1; done
