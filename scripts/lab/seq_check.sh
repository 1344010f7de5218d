#!/bin/bash
# The sequence tests and bench lines after a sequence-kernel change (results under gpurun_out/).
export TMPDIR=/tmp; mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "sequence or front_half or rmat_generator or knobs_exact or multi" > gpurun_out/pytest_seq.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/pytest_seq.log; exit 1; }
tail -1 gpurun_out/pytest_seq.log
for r in 1 2; do
  $T 150 python bench.py --no-cpu-baseline > gpurun_out/b26_$r.json 2> gpurun_out/b26_$r.err || exit 1
done
$T 150 python bench.py --no-cpu-baseline --scale 22 --seed 22 --check > gpurun_out/b22.json 2>&1 || exit 1
$T 150 python bench.py --no-cpu-baseline --workload twitter > gpurun_out/btw.json 2>&1 || exit 1
$T 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1 || { echo prof_fail; exit 1; }
echo all_ok
