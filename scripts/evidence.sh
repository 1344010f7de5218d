#!/bin/bash
# A round's evidence for HEAD under $OUT: the default bench line (with both CPU baselines), the
# LJ / twitter / RMAT-22 lines, rocprofv3 kernel stats of the headline run (4 timed steps +
# 1 warmup), and FETCH_SIZE / WRITE_SIZE in separate --pmc passes over one step.
set -o pipefail
OUT=${OUT:-gpurun_out/ev}
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$OUT/bench_rmat26.json" 2> "$OUT/bench.err" && echo "bench ok" &&
timeout -k 10 200 python bench.py --workload lj --no-cpu-baseline > "$OUT/bench_lj.json" 2>> "$OUT/bench.err" && echo "lj ok" &&
timeout -k 10 200 python bench.py --workload twitter --no-cpu-baseline > "$OUT/bench_twitter.json" 2>> "$OUT/bench.err" && echo "tw ok" &&
timeout -k 10 200 python bench.py --scale 22 --seed 22 --no-cpu-baseline --check > "$OUT/bench_rmat22_checked.json" 2>> "$OUT/bench.err" && echo "rmat22 ok" &&
rm -rf "$OUT/prof" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 && echo "prof ok" &&
rm -rf "$OUT/pmc/fetch" && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc/fetch" -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc/fetch.log" 2>&1 && echo "fetch ok" &&
rm -rf "$OUT/pmc/write" && timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc/write" -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc/write.log" 2>&1 && echo "write ok"
