set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --steps 20 > gpurun_out/m_serial.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --steps 20 --mc-beside-ms > gpurun_out/m_tail.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --steps 20 --concurrent > gpurun_out/m_conc.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --steps 20 --mc-beside-ms > gpurun_out/m_tail2.log 2>&1
rc=$?
for f in gpurun_out/m_serial.log gpurun_out/m_tail.log gpurun_out/m_conc.log gpurun_out/m_tail2.log; do
  python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['per_kernel_ms'].items()}, d['config']['streams'])" 2>/dev/null
done
exit $rc
