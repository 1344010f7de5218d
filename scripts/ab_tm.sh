#!/bin/bash
# A/B of the tile-major bin counts (SHEEP_BIN_TM): parity tests, checked RMAT-22, RMAT-26 both ways.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 400 python bench.py --scale 22 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/bench22.log 2>&1 && echo "bench22 ok" &&
SHEEP_BIN_TM=0 timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench26_tm0.log 2>&1 && echo "tm0 ok" &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench26_tm1.log 2>&1 && echo "tm1 ok" &&
timeout -k 10 400 python bench.py --workload lj --steps 5 --warmup 2 --no-cpu-baseline --check > gpurun_out/benchlj.log 2>&1 && echo "lj ok"
