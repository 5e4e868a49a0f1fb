#!/bin/bash
# PMC passes over bench.py (one counter group per rocprofv3 run, no tracing domains combined
# with --pmc).  Output: gpurun_out/pmc/<pass>/..._counter_collection.csv + <pass>.log.
# Usage: tools/pmc.sh [pass ...]   (default: all passes)
export TMPDIR=/tmp
# PMC_BENCH / PMC_OUT / PMC_TRAFFIC / PMC_CONFIG select another workload (e.g. tools/bench_lines.py)
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
BENCH=${PMC_BENCH:-"python3 bench.py --steps 3 --warmup 1 --settle-steps 2 --no-cpu"}
declare -A P
P[sq1]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P[sq2]="SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P[tcp]="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum"
P[lat]="SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH"
P[sqc]="SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_DCACHE_REQ SQC_TC_DATA_READ_REQ SQC_TC_STALL"
P[lat2]="SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_INSTS_VMEM_WR SQ_INSTS_SMEM_NORM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
P[icache]="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
P[fetch]="FETCH_SIZE"
P[write]="WRITE_SIZE"
passes=("$@")
[ ${#passes[@]} -eq 0 ] && passes=(sq1 sq2 fetch write)
for p in "${passes[@]}"; do
  echo "=== pmc pass $p: ${P[$p]}"
  # shellcheck disable=SC2086
  timeout -k 10 300 rocprofv3 --pmc ${P[$p]} -d "$OUT/$p" -o "$p" --output-format csv -- $BENCH > "$OUT/$p.log" 2>&1
  rc=$?
  echo "=== pmc pass $p rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$p.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT"
python3 tools/pmc_traffic.py "$OUT" "${PMC_TRAFFIC:-gpurun_out/pmc_traffic.json}" > /dev/null
