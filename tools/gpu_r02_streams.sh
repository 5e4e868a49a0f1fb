# serial vs one-stream-per-kind step on one MI355X (each run under its own limit)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --steps 20 > gpurun_out/r02_bench_streams.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --steps 20 --serial > gpurun_out/r02_bench_serial.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --steps 20 > gpurun_out/r02_bench_streams2.log 2>&1
rc=$?
for f in gpurun_out/r02_bench_streams.log gpurun_out/r02_bench_serial.log gpurun_out/r02_bench_streams2.log; do
  python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['per_kernel_ms'].items()}, round(d['group_ms'],3))"
done
exit $rc
