# whole -m gpu suite + smoke, then the phase profile (SDX_PROF build) of the grouped k_pulses.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02_gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && \
SDX_LIB=pysignalduino_amd/_lib/variants/libsdx_prof.so timeout -k 10 120 python -u tools/prof_phases.py > gpurun_out/r02_phase_prof_grouped.log 2>&1
rc=$?
tail -3 gpurun_out/r02_gpu_tests.log; tail -2 gpurun_out/r02_smoke.log 2>/dev/null; cat gpurun_out/r02_phase_prof_grouped.log 2>/dev/null | tail -30
exit $rc
