#!/bin/bash
# Round 6 evidence for HEAD, ONE lease (the line's roofline must reproduce
# from the same lease's profiles): the GPU suite; the default bench line (both CPU baselines);
# the LJ / twitter / RMAT-22 (checked) lines; rocprofv3 kernel stats of the headline (4 timed
# steps + 1 warmup); the PMC passes of one step (FETCH_SIZE, WRITE_SIZE, TCC hit / miss /
# atomics, LDS, waves: one --pmc run each).  Everything under $OUT.  (The one-rank RCCL driver
# line and the P = 8 lockstep simulation: scripts/evidence_r06_multi.sh, a lease of its own.)
set -o pipefail
OUT=${OUT:-gpurun_out/ev_r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py > "$OUT/bench_rmat26.json" 2> "$OUT/bench.err" && echo "bench ok" &&
timeout -k 10 200 python bench.py --workload lj --no-cpu-baseline > "$OUT/bench_lj.json" 2>> "$OUT/bench.err" && echo "lj ok" &&
timeout -k 10 200 python bench.py --workload twitter --no-cpu-baseline > "$OUT/bench_twitter.json" 2>> "$OUT/bench.err" && echo "tw ok" &&
timeout -k 10 200 python bench.py --scale 22 --seed 22 --no-cpu-baseline --check > "$OUT/bench_rmat22_checked.json" 2>> "$OUT/bench.err" && echo "rmat22 ok" &&
rm -rf "$OUT/prof" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 && echo "prof ok" &&
OUT="$OUT/pmc" PASSES="fetch write tcc lds wave" bash scripts/pmc_r04.sh
