# Round 6: the fault word's address cached per device (hipGetSymbolAddress once): bench lines of
# the four configs and the LJ / RMAT-26 step gaps.
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "known or hep or corrupt or walk_guard or range" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
OUT=$O TESTS=0 bash scripts/gpu_round.sh || exit 1
for w in "--workload lj" "--scale 26"; do
  n=$(echo $w | tr -d ' -')
  rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py $w --steps 2 --warmup 1 --no-cpu-baseline > $O/tr_$n.log 2>&1 || exit 1
  f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
  python scripts/step_gaps.py $f > $O/${n}_step_gaps.txt; rm -rf $O/tr
done
