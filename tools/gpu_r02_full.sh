# round-2 check: the whole -m gpu suite, smoke, then the default bench and the per-kind benches.
# Each GPU step runs under its own time limit; the chain stops at the first failure.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/r02_bench_mixed.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MU --no-cpu > gpurun_out/r02_bench_mu.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MU --corpus dense --no-cpu > gpurun_out/r02_bench_mu_dense.log 2>&1
rc=$?
tail -3 gpurun_out/r02_gpu_tests.log; tail -1 gpurun_out/r02_bench_mixed.log gpurun_out/r02_bench_mu.log gpurun_out/r02_bench_mu_dense.log 2>/dev/null
exit $rc
