# general path: parity tests, then the timing of the general goldens (tools/time_general.py)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_general.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02_general.log 2>&1 && \
timeout -k 10 240 python -u tools/time_general.py > gpurun_out/r02_time_general.log 2>&1
rc=$?
tail -4 gpurun_out/r02_general.log; cat gpurun_out/r02_time_general.log
exit $rc
