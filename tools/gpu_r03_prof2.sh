#!/bin/bash
# phase + per-group profile (SDX_PROF build), and the default bench's kernel trace (gaps per step)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_prof2}
mkdir -p "$O"
SDX_LIB=pysignalduino_amd/_lib/variants/libsdx_prof.so timeout -k 10 120 python -u tools/prof_phases.py > "$O/phase_prof.log" 2>&1 || { tail -20 "$O/phase_prof.log"; exit 1; }
grep -v amdgpu.ids "$O/phase_prof.log"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/kt" -o b --output-format csv -- \
  python3 bench.py --no-cpu --steps 10 > "$O/bench.log" 2>&1 || { tail -30 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-200
