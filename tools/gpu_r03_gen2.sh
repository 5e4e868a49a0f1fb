set -u -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/gen1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_general.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 200 python tools/time_general.py > $O/time.log 2>&1 || { tail -20 $O/time.log; exit 1; }
cat $O/time.log
SDX_LIB=pysignalduino_amd/_lib/variants/libsdx_gprof.so timeout -k 10 200 python tools/prof_general.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cat $O/prof.log
