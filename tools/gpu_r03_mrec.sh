#!/bin/bash
# Round 3: message records (sdx_msg_rec) -- the whole -m gpu suite, bench A/B against --no-mrec,
# PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of both.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/r03_mrec
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > "$O/tests.txt" 2>&1 \
  || { tail -60 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for r in 1 2; do
  for m in "" "--mrec"; do
    timeout -k 10 180 python bench.py --no-cpu $m > "$O/b.log" 2>&1 || { tail -30 "$O/b.log"; exit 1; }
    python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print('mode=$m',round(d['value']/1e6,1),{k:round(v,3) for k,v in d['per_kernel_ms'].items()},round(d['ms_per_step'],3))" | tee -a "$O/ab.log"
  done
done
PMC_OUT=$O/pmc PMC_TRAFFIC=$O/pmc_traffic_mrec.json bash tools/pmc.sh fetch write > "$O/pmc.log" 2>&1 || { tail -30 "$O/pmc.log"; exit 1; }
PMC_BENCH="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-mrec" PMC_OUT=$O/pmc_soa PMC_TRAFFIC=$O/pmc_traffic_soa.json \
  bash tools/pmc.sh fetch write > "$O/pmc_soa.log" 2>&1 || { tail -30 "$O/pmc_soa.log"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for tag in ("mrec", "soa"):
    d = json.load(open(f"{o}/pmc_traffic_{tag}.json"))
    print(tag, {k: (round(v["fetch_size_kib"] / 1024, 1), round(v["write_size_kib"] / 1024, 1), round(v["traffic_bytes"] / 1e6, 1))
                for k, v in d.items() if not k.startswith("_")})
PY
