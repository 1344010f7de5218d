#!/bin/bash
# PMC passes over one RMAT-26 step (sequential kb loop), summary per kernel in gpurun_out/pmc/*
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp SHEEP_KB_PIPE=0
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1)); rm -rf gpurun_out/pmc/p$i
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/b$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
