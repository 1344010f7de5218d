#!/bin/bash
# Tree-phase lab on one box: per-bucket statistics of one RMAT-26 build (SHEEP_TREE_STATS=2:
# unpipelined, counters on; stderr lines "bucket k ranks [..) edges .. kept .. finds .. zip ..
# steps .. cas .."), then A/B of the bucket-merge lab option on the four bench configs.
#   OUT=gpurun_out/tree bash scripts/tree_lab.sh
set -o pipefail
OUT=${OUT:-gpurun_out/tree}
mkdir -p "$OUT"
SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
  > "$OUT/stats_rmat26.json" 2> "$OUT/stats_rmat26.txt" && echo "stats ok" &&
OUT=$OUT bash scripts/ab_env.sh "--steps 8 --warmup 2 --no-cpu-baseline" - SHEEP_KB_MERGE=20 SHEEP_KB_MERGE=50 SHEEP_KB_MERGE=100 - &&
OUT=$OUT bash scripts/ab_env.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" - SHEEP_KB_MERGE=20 SHEEP_KB_MERGE=50 SHEEP_KB_MERGE=100 &&
OUT=$OUT bash scripts/ab_env.sh "--scale 22 --seed 22 --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_KB_MERGE=20 SHEEP_KB_MERGE=50 SHEEP_KB_MERGE=100 &&
OUT=$OUT bash scripts/ab_env.sh "--workload lj --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_KB_MERGE=20 SHEEP_KB_MERGE=50 SHEEP_KB_MERGE=100
