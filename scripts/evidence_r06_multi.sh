#!/bin/bash
# Round 6, multi-rank evidence at HEAD: the C++ multi-rank driver over a one-rank RCCL group
# (bench.py --lockstep-1) beside the single path on the same box, and the P = 8 lockstep
# simulation (scripts/lockstep_sim.py: 8 shards as 8 sessions on one GPU, bit-exact).
set -o pipefail
OUT=${OUT:-gpurun_out/ev_r06_multi}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/single_$i.json" 2>> "$OUT/bench.err" &&
  timeout -k 10 200 python bench.py --lockstep-1 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/lockstep1_$i.json" 2>> "$OUT/bench.err" || exit 1
  echo "pair $i ok"
done
timeout -k 10 500 python scripts/lockstep_sim.py --P 8 --reps 2 > "$OUT/sim.jsonl" 2> "$OUT/sim.err" && echo "sim ok"
