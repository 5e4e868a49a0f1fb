#!/bin/bash
# Round 3: phase profiles (SDX_PROF builds: SWAR staging vs the ballot staging), then the whole
# suite + benches (tools/gpu_r03_all.sh).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r03_prof}
mkdir -p "$O"
V=pysignalduino_amd/_lib/variants
SDX_LIB=$V/libsdx_prof.so timeout -k 10 120 python -u tools/prof_phases.py > "$O/phase_prof_swar.log" 2>&1 || { tail -20 "$O/phase_prof_swar.log"; exit 1; }
SDX_LIB=$V/libsdx_profballot.so timeout -k 10 120 python -u tools/prof_phases.py > "$O/phase_prof_ballot.log" 2>&1 || { tail -20 "$O/phase_prof_ballot.log"; exit 1; }
grep -v amdgpu.ids "$O/phase_prof_swar.log"
[ "${2:-all}" = "all" ] && bash tools/gpu_r03_all.sh "${1:-r03_prof}_all"
