# general path (multi-digit ids, long messages / frames) on the GPU, then the whole -m gpu suite.
# Each GPU step under its own time limit; the chain stops at the first failure.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_general.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02_general.log 2>&1 && \
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1
rc=$?
tail -5 gpurun_out/r02_general.log; tail -3 gpurun_out/r02_gpu_tests.log 2>/dev/null; tail -2 gpurun_out/r02_smoke.log 2>/dev/null
exit $rc
