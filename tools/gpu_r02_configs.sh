# configs 2-4 at their stated size (1M of one kind) and the dense MU corpus, one MI355X
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --kind MU --no-cpu > gpurun_out/c_mu.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MS --no-cpu > gpurun_out/c_ms.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MC --no-cpu > gpurun_out/c_mc.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MU --corpus dense --no-cpu > gpurun_out/c_mu_dense.log 2>&1
rc=$?
for f in gpurun_out/c_mu.log gpurun_out/c_ms.log gpurun_out/c_mc.log gpurun_out/c_mu_dense.log; do
  python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['per_kernel_ms'].items()}, round(d['roofline']['frac'],5), d.get('overflow'))" 2>/dev/null
done
exit $rc
