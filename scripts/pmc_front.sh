#!/bin/bash
# PMC passes over the front-half kernels of one RMAT-26 graph2tree (scripts/map_lab.py):
# one rocprofv3 --pmc run per counter group (hardware limits per pass), CSV under $OUT.
set -e
OUT=${OUT:-gpurun_out/pmc_front}
RE=${RE:-"k_part|k_degb|k_edge_pass|k_bin_scatter"}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
         "FETCH_SIZE" \
         "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
         "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$RE" --output-format csv \
    -d "$OUT/p$i" -o p -- python scripts/map_lab.py --reps 1 ${LAB_ARGS} > "$OUT/p$i.log" 2>&1
  echo "pass $i done"
done
