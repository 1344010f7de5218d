#!/bin/bash
# A/B of the counting-sort sequence (seq_sort 2) and the y-ordered second partition pass
# (part_ysort) at RMAT-26 and RMAT-22, after their parity tests.  Run from the repo root on
# the GPU box; results under gpurun_out/.
export TMPDIR=/tmp; mkdir -p gpurun_out
T="timeout -k 10"
$T 240 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "sequence_from_degrees or front_half" > gpurun_out/pytest_seq.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/pytest_seq.log; exit 1; }
tail -1 gpurun_out/pytest_seq.log
SHEEP_SEQ_SORT=2 $T 240 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "front_half or rmat_generator or knobs_exact" > gpurun_out/pytest_seq2.log 2>&1 || { echo tests2_fail; tail -30 gpurun_out/pytest_seq2.log; exit 1; }
tail -1 gpurun_out/pytest_seq2.log
for rep in 1 2; do
 for cfg in "26 26" "22 22"; do set -- $cfg
  [ $rep = 2 ] && [ $1 = 22 ] && continue
  for v in "base:SHEEP_SEQ_SORT=1" "seq2:SHEEP_SEQ_SORT=2" "ys0:SHEEP_PART_YSORT=0"; do n=${v%%:*}; e=${v#*:}
   env $e $T 150 python bench.py --no-cpu-baseline --scale $1 --seed $2 > gpurun_out/ab_${1}_${n}_$rep.json 2> gpurun_out/ab_${1}_${n}_$rep.err || { echo bench_fail $1 $n; exit 1; }
  done
 done
done
echo benches_ok
