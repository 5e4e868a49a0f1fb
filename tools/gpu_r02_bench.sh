# round-2 bench variants on one MI355X (each step under its own time limit; stop at the first failure)
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -m pytest tests/test_dist.py tests/test_units.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_gpu_dist_units.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/r02_bench_mixed.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MU --no-cpu > gpurun_out/r02_bench_mu.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MS --no-cpu > gpurun_out/r02_bench_ms.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MC --no-cpu > gpurun_out/r02_bench_mc.log 2>&1 && \
timeout -k 10 200 python bench.py --kind MU --corpus dense --no-cpu > gpurun_out/r02_bench_mu_dense.log 2>&1 && \
SDX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --msgs 300000 --no-cpu > gpurun_out/r02_gloo2.log 2>&1
