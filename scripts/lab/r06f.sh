# Round 6: the edge pass over a tile map of the x-digit regions (no per-tile digit search):
# the GPU suite, then bench lines alternating with the library before it (base = HEAD 542723d
# build with the cached walk-guard address), then the inter-call gaps of LJ / RMAT-26.
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --no-cpu-baseline --steps 20 --warmup 3" 1 || exit 1
for w in "--workload lj" "--scale 26"; do
  n=$(echo $w | tr -d ' -')
  rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py $w --steps 3 --warmup 1 --no-cpu-baseline > $O/tr_$n.log 2>&1 || exit 1
  f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
  python scripts/step_gaps.py --prev $f > $O/${n}_prev_step_gaps.txt; rm -rf $O/tr
done
