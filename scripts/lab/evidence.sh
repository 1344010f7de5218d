#!/bin/bash
# Round evidence at HEAD: the GPU suite, smoke, the four bench configs (RMAT-22 checked) and a
# rocprofv3 kernel-stats pass of the default bench.  Results under gpurun_out/.
export TMPDIR=/tmp; mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo suite_fail; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
$T 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; tail gpurun_out/smoke.log; exit 1; }
echo smoke_ok
$T 300 python bench.py > gpurun_out/bench_rmat26.json 2> gpurun_out/bench_rmat26.err || exit 1
$T 150 python bench.py --no-cpu-baseline --scale 22 --seed 22 --check > gpurun_out/bench_rmat22_checked.json 2>&1 || exit 1
$T 150 python bench.py --no-cpu-baseline --workload lj > gpurun_out/bench_lj.json 2>&1 || exit 1
$T 200 python bench.py --no-cpu-baseline --workload twitter > gpurun_out/bench_twitter.json 2>&1 || exit 1
echo benches_ok
$T 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof_fail; tail gpurun_out/prof.log; exit 1; }
echo prof_ok
