set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_units.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02_units.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1
