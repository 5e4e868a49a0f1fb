set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/pcs
timeout -k 10 120 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1 || echo "list rc $?"
grep -i -B2 -A12 "pc.sampl" gpurun_out/pcs/list.txt | head -60
SDX_KINDS=MU timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d gpurun_out/pcs/run -o mu -- python3 tools/time_mu.py 333333 3 > gpurun_out/pcs/run.log 2>&1
echo "rc $?"
tail -5 gpurun_out/pcs/run.log
find gpurun_out/pcs -type f | head; 
