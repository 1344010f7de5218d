#!/bin/bash
# Round-4 counter evidence for one RMAT-26 graph2tree step (bench.py --steps 1 --warmup 0):
# one rocprofv3 --pmc run per counter group (MI355X_MICROARCH.md: separate passes, at most
# 4 TCC / 8 SQ counters each), CSVs under $OUT/<pass>.  scripts/pmc_r04_table.py turns them into
# the per-kernel table (bytes, L2 hit rate, atomics, LDS conflicts, time).
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_r04}
ARGS=${ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline"}
PASSES=${PASSES:-"fetch write tcc lds wave"}
mkdir -p "$OUT"
export TMPDIR=/tmp
for P in $PASSES; do
  case $P in
    fetch) C="FETCH_SIZE" ;;
    write) C="WRITE_SIZE" ;;
    tcc) C="TCC_HIT_sum TCC_MISS_sum TCC_ATOMIC_sum" ;;
    tccreq) C="TCC_REQ_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" ;;
    lds) C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" ;;
    wave) C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" ;;
    *) echo "unknown pass $P"; exit 2 ;;
  esac
  rm -rf "$OUT/$P"
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/$P" -o run -- \
    python bench.py $ARGS > "$OUT/$P.log" 2>&1 || { echo "pass $P failed"; exit 1; }
  echo "pass $P done"
done
