#!/bin/bash
# A round's evidence for HEAD under $OUT: the default bench line (with both CPU baselines), the
# LJ / twitter / RMAT-22 lines, rocprofv3 kernel stats of the headline run (4 timed steps +
# 1 warmup), the counter passes of scripts/pmc_r04.sh over one step (FETCH_SIZE, WRITE_SIZE,
# TCC hit / miss / atomics, LDS, waves: one --pmc run each), and the front half's phases in five
# separate processes (scripts/lab/front_var.py: the run-to-run spread).
set -o pipefail
OUT=${OUT:-gpurun_out/ev}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$OUT/bench_rmat26.json" 2> "$OUT/bench.err" && echo "bench ok" &&
timeout -k 10 200 python bench.py --workload lj --no-cpu-baseline > "$OUT/bench_lj.json" 2>> "$OUT/bench.err" && echo "lj ok" &&
timeout -k 10 200 python bench.py --workload twitter --no-cpu-baseline > "$OUT/bench_twitter.json" 2>> "$OUT/bench.err" && echo "tw ok" &&
timeout -k 10 200 python bench.py --scale 22 --seed 22 --no-cpu-baseline --check > "$OUT/bench_rmat22_checked.json" 2>> "$OUT/bench.err" && echo "rmat22 ok" &&
rm -rf "$OUT/prof" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 && echo "prof ok" &&
OUT="$OUT/pmc" PASSES="fetch write tcc lds wave" bash scripts/pmc_r04.sh &&
for i in 1 2 3 4 5; do
  timeout -k 10 120 python scripts/lab/front_var.py --reps 4 >> "$OUT/front_var.jsonl" 2>> "$OUT/front_var.err" || exit 1
  echo "front_var $i ok"
done
