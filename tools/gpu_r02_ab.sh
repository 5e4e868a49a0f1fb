# parity (MU/MS kernels) then two 20-step bench runs (serial launches)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_units.py tests/test_general.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_ab_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --steps 20 > gpurun_out/r02_ab_1.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --steps 20 > gpurun_out/r02_ab_2.log 2>&1
rc=$?
tail -2 gpurun_out/r02_ab_tests.log
for f in gpurun_out/r02_ab_1.log gpurun_out/r02_ab_2.log; do
  python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['per_kernel_ms'].items()}, round(d['group_ms'],3))" 2>/dev/null
done
exit $rc
