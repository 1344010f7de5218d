#!/bin/bash
# One GPU round trip for a build: the -m gpu suite (optional), then the four bench lines
# (RMAT-26 headline, RMAT-22 checked against the CPU checker, LJ and twitter shapes), each
# under its own time limit, chained so that the first failure ends the call.
#   OUT=gpurun_out/x TESTS=1 bash scripts/gpu_round.sh
set -o pipefail
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_rmat26.json" 2>> "$OUT/bench.err" && echo "rmat26 ok" &&
timeout -k 10 240 python bench.py --scale 22 --seed 22 --no-cpu-baseline --check --steps 20 --warmup 3 > "$OUT/bench_rmat22_checked.json" 2>> "$OUT/bench.err" && echo "rmat22 ok" &&
timeout -k 10 240 python bench.py --workload lj --no-cpu-baseline --steps 20 --warmup 3 > "$OUT/bench_lj.json" 2>> "$OUT/bench.err" && echo "lj ok" &&
timeout -k 10 240 python bench.py --workload twitter --no-cpu-baseline --steps 6 --warmup 2 > "$OUT/bench_twitter.json" 2>> "$OUT/bench.err" && echo "twitter ok"
