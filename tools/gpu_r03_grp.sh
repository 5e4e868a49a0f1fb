set -u -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/grp
timeout -k 10 200 python tools/exp_group_cost.py > gpurun_out/grp/exp.log 2>&1 || { tail -20 gpurun_out/grp/exp.log; exit 1; }
tail -4 gpurun_out/grp/exp.log
for r in 1 2; do for f in "" "--concurrent"; do
 timeout -k 10 180 python bench.py --no-cpu $f > gpurun_out/grp/b$r$f.log 2>&1 || exit 1
 echo "$f $r: $(tail -1 gpurun_out/grp/b$r$f.log | cut -c80-160)"; done; done
