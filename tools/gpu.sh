#!/bin/bash
# One parameterised GPU-box script (replaces the per-experiment gpu_r0*_*.sh of rounds 2-3).
#   tools/gpu.sh OUT STEP [STEP ...]        (run from the repo root, e.g. through gpurun)
# Every step has its own time limit; the script stops at the first failure (no retries).
# Steps:
#   testc[=PYTEST_K]     like tests but without -x, and the script goes on after test FAILURES
#                        (not after a timeout, abort or crash: exit status 124/134/137/139 stops it)
#   warm                 import torch + device name (a fresh box pages torch in: 1-2 min)  -> OUT/warm.log
#   tests[=PYTEST_K]     the whole -m gpu suite (or -k PYTEST_K)            -> OUT/tests*.txt
#   smoke                __graft_entry__.smoke()                           -> OUT/smoke.log
#   bench[=ARGS]         python bench.py ARGS (',' separates arguments)    -> OUT/bench_<n>.log
#   benchcpu             bench.py with the cpu_baseline leg                -> OUT/bench_cpu.log
#   lines[=ARGS]         tools/bench_lines.py --no-cpu ARGS                -> OUT/lines_<n>.log
#   e2e[=ARGS]           tools/bench_lines_e2e.py --check ARGS             -> OUT/e2e_<n>.log
#   kt                   rocprofv3 --kernel-trace --stats of bench.py      -> OUT/kt_bench/
#   ktlines              the same for tools/bench_lines.py                 -> OUT/kt_lines/
#   ktpy=SCRIPT[,ARGS]   the same for python3 SCRIPT ARGS                  -> OUT/kt_<n>/
#   ktpyenv=VAR=val,SCRIPT[,ARGS]  the same with VAR=val in the environment -> OUT/kt_<n>/
#   ktx[=ARGS]           the same for bench.py --no-cpu ARGS (',' separates) -> OUT/ktx_<n>/
#   pmc[=PASSES]         tools/pmc.sh (default sq1,sq2,fetch,write)        -> OUT/pmc/, OUT/pmc_traffic.json
#   time=V1,V2           tools/time_mu.py for in-tree libsdx + variants V (pysignalduino_amd/_lib/ab/libsdx_V.so), 2 rounds
#   env=E1,E2            bench.py --no-cpu under env settings E (VAR=value), 2 rounds
#   py=SCRIPT[,ARGS]     python SCRIPT ARGS (a tools/ measurement)          -> OUT/py_<n>.log
#   benchenv=VAR=val[,ARGS]  bench.py ARGS with VAR=val in the environment -> OUT/bench_<n>.log
#   pyenv=VAR=val,SCRIPT[,ARGS]  python SCRIPT ARGS with VAR=val in the environment -> OUT/pyenv_<n>.log
#   pylib=V,SCRIPT[,ARGS] the same with SDX_LIB = pysignalduino_amd/_lib/ab/libsdx_V.so (e.g. the SDX_PROF build)
#   testlib=V[,PYTEST_K]  the -m gpu suite (or -k) on the variant library V (like testc)
#   benchlib=V[,ARGS]     bench.py ARGS on the variant library V
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O=gpurun_out/$1; shift; mkdir -p "$O"
n=0
summ() { python3 -c 'import json,sys
for ln in sys.stdin:
    pass
try:
    d=json.loads(ln)
    print(round(d["value"]/1e6,2), "M", d.get("unit","")+",", round(d.get("ms_per_step",0),4), "ms/step", {k: round(v,4) for k,v in d.get("per_kernel_ms",{}).items()})
except Exception:
    print(ln[:300].rstrip())'; }
run() {  # run LIMIT LOG CMD...: the step's output to LOG, its tail on failure
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1 || { echo "FAILED ($?): $*"; tail -40 "$log"; exit 1; }
}
for st in "$@"; do
  n=$((n+1)); name=${st%%=*}; arg=""; [ "$name" != "$st" ] && arg=${st#*=}
  args=${arg//,/ }
  case $name in
    warm) run 240 "$O/warm.log" python -u -c "print('importing torch', flush=True); import torch; print(torch.cuda.get_device_name(0), flush=True)"
      tail -1 "$O/warm.log" ;;
    testc)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v ${arg:+-k "$arg"} --timeout 150 --timeout-method thread > "$O/testc_$n.txt" 2>&1
      rc=$?
      tail -1 "$O/testc_$n.txt"
      grep -E "^(FAILED|ERROR)" "$O/testc_$n.txt" | head -20 || true
      case $rc in 124|134|137|139) echo "tests stopped ($rc): no further GPU steps"; exit 1 ;; esac ;;
    tests)
      if [ -n "$arg" ]; then run 900 "$O/tests_$n.txt" python -u -m pytest tests -m gpu -x -v -k "$arg" --timeout 150 --timeout-method thread
      else run 900 "$O/tests.txt" python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread; fi
      tail -1 "$O"/tests*.txt | tail -1 ;;
    smoke) run 240 "$O/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"; tail -1 "$O/smoke.log" ;;
    bench) run 240 "$O/bench_$n.log" python bench.py --no-cpu $args; echo "bench $arg: $(tail -1 "$O/bench_$n.log" | summ)" ;;
    benchcpu) run 360 "$O/bench_cpu.log" python bench.py; tail -1 "$O/bench_cpu.log" | cut -c1-400 ;;
    lines) run 300 "$O/lines_$n.log" python tools/bench_lines.py --no-cpu $args; echo "lines $arg: $(tail -1 "$O/lines_$n.log" | cut -c1-300)" ;;
    e2e) run 400 "$O/e2e_$n.log" python -u tools/bench_lines_e2e.py --check $args; echo "e2e $arg: $(tail -1 "$O/e2e_$n.log" | cut -c1-400)" ;;
    kt) run 300 "$O/kt_bench.log" rocprofv3 --kernel-trace --stats -d "$O/kt_bench" -o b --output-format csv -- python3 bench.py --no-cpu
        echo "kt: $(tail -1 "$O/kt_bench.log" | summ)" ;;
    ktpy) run 300 "$O/ktpy_$n.log" rocprofv3 --kernel-trace --stats -d "$O/kt_$n" -o k --output-format csv -- python3 $args
        echo "ktpy $arg: $(tail -1 "$O/ktpy_$n.log" | cut -c1-300)" ;;
    ktpyenv) e=${args%% *}; rest=${args#* }
      run 300 "$O/ktpyenv_$n.log" env "$e" rocprofv3 --kernel-trace --stats -d "$O/kt_$n" -o k --output-format csv -- python3 $rest
      echo "ktpyenv $arg: $(tail -3 "$O/ktpyenv_$n.log" | cut -c1-300)" ;;
    ktx) run 300 "$O/ktx_$n.log" rocprofv3 --kernel-trace --stats -d "$O/ktx_$n" -o b --output-format csv -- python3 bench.py --no-cpu $args
        echo "ktx $arg: $(tail -1 "$O/ktx_$n.log" | summ)" ;;
    ktlines) run 300 "$O/kt_lines.log" rocprofv3 --kernel-trace --stats -d "$O/kt_lines" -o l --output-format csv -- python3 tools/bench_lines.py --no-cpu
        echo "ktlines: $(tail -1 "$O/kt_lines.log" | cut -c1-200)" ;;
    pmc) PMC_OUT=$O/pmc PMC_TRAFFIC=$O/pmc_traffic.json run 1200 "$O/pmc.log" bash tools/pmc.sh ${args:-sq1 sq2 fetch write}
        tail -14 "$O/pmc.log" ;;
    time)
      for r in 1 2; do for v in base $args; do
        if [ "$v" = base ]; then L=""; else L=pysignalduino_amd/_lib/ab/libsdx_$v.so; fi
        SDX_LIB=$L run 150 "$O/time_${v}_$r.log" python tools/time_mu.py
        echo "time $v $r: $(tail -1 "$O/time_${v}_$r.log")"
      done; done ;;
    env)
      for r in 1 2; do for e in $args; do
        tag=$(echo "$e" | tr '=/ ' '___')
        run 240 "$O/env_${tag}_$r.log" env "$e" python bench.py --no-cpu
        echo "$e $r: $(tail -1 "$O/env_${tag}_$r.log" | summ)"
      done; done ;;
    py) run 600 "$O/py_$n.log" python -u $args; echo "py $arg: $(tail -3 "$O/py_$n.log" | cut -c1-400)" ;;
    benchenv) e=${args%% *}; rest=${args#* }; [ "$rest" = "$e" ] && rest=""
      run 240 "$O/bench_$n.log" env "$e" python bench.py --no-cpu $rest
      echo "bench $arg: $(tail -1 "$O/bench_$n.log" | summ)" ;;
    pyenv) e=${args%% *}; rest=${args#* }
      run 600 "$O/pyenv_$n.log" env "$e" python -u $rest
      echo "pyenv $arg: $(tail -3 "$O/pyenv_$n.log" | cut -c1-400)" ;;
    pylib) v=${args%% *}; rest=${args#* }
      SDX_LIB=pysignalduino_amd/_lib/ab/libsdx_$v.so run 600 "$O/pylib_$n.log" python -u $rest
      echo "pylib $arg: $(tail -3 "$O/pylib_$n.log" | cut -c1-400)" ;;
    testlib) v=${args%% *}; k=${args#* }; [ "$k" = "$v" ] && k=""
      SDX_LIB=pysignalduino_amd/_lib/ab/libsdx_$v.so timeout -k 10 900 python -u -m pytest tests -m gpu -v ${k:+-k "$k"} --timeout 150 --timeout-method thread > "$O/testlib_$n.txt" 2>&1
      rc=$?
      echo "testlib $arg: $(tail -1 "$O/testlib_$n.txt")"
      grep -E "^(FAILED|ERROR)" "$O/testlib_$n.txt" | head -20 || true
      case $rc in 124|134|137|139) echo "tests stopped ($rc): no further GPU steps"; exit 1 ;; esac ;;
    benchlib) v=${args%% *}; rest=${args#* }; [ "$rest" = "$v" ] && rest=""
      SDX_LIB=pysignalduino_amd/_lib/ab/libsdx_$v.so run 240 "$O/bench_$n.log" python bench.py --no-cpu $rest
      echo "benchlib $arg: $(tail -1 "$O/bench_$n.log" | summ)" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "gpu.sh done"
