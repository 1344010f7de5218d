#!/bin/bash
# PMC passes over the front-half kernels of one RMAT-26 bench step (one rocprofv3 --pmc run per
# counter group: the hardware limits per pass), CSV under $OUT.
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_fh}
RE=${RE:-"k_fh|k_degb|k_part|k_edge_bin|k_tm_"}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i + 1))
  rm -rf "$OUT/p$i"
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$RE" --output-format csv \
    -d "$OUT/p$i" -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/p$i.log" 2>&1 || exit $?
  echo "pass $i done"
done
