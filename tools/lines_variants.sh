#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for spec in "1,1,1:0.3" "1,1,1:0" "1,0,0:0" "1,0,0:1" "0,1,0:0" "0,1,0:1" "0,0,1:0"; do
  mix=${spec%%:*}; cf=${spec##*:}
  timeout -k 10 200 python3 tools/bench_lines.py --no-cpu --steps 3 --warmup 1 --mix $mix --compress-frac $cf > /tmp/v.log 2>&1 || { tail -5 /tmp/v.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('/tmp/v.log').read().strip().splitlines()[-1]); k=d['per_kernel_ms']
print('$mix cf=$cf parse %.3f ms  MU %.3f MS %.3f MC %.3f  bytes %d' % (k['parse'], k['MU'], k['MS'], k['MC'], d['config']['line_bytes']))"
done
