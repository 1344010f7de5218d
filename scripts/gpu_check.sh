#!/bin/bash
# One GPU session: parity tests, smoke, a checked small bench, the headline bench, a rocprof
# kernel trace.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE=${SCALE:-26}
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py --scale 22 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/bench22.log 2>&1 && echo "bench22 ok" &&
timeout -k 10 600 python bench.py --scale $SCALE --steps 5 --warmup 2 > gpurun_out/bench26.log 2>&1 && echo "bench26 ok" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --scale $SCALE --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && echo "prof ok"
