# Round 6: (1) the refresh makes the zipper's first step of the pairs from pre-bucket roots
# (SHEEP_KB_RLINK=1, new default): the GPU suite, then bench lines alternating 1 / 0;
# (2) the tile-mapped second partition pass (HEAD with SHEEP_KB_RLINK=0) against the library at
# 304d53e (base), alternating on this box; (3) the RMAT-26 kb timeline and kernel traces of
# RMAT-26 / twitter / LJ at HEAD.
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_KB_RLINK=0 - SHEEP_KB_RLINK=0 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_KB_RLINK=0 - SHEEP_KB_RLINK=0 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_KB_RLINK=0 - SHEEP_KB_RLINK=0 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_KB_RLINK=0 || exit 1
SHEEP_KB_RLINK=0 OUT=$O/tilemap bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 2 || exit 1
SHEEP_KB_RLINK=0 OUT=$O/tilemap bash scripts/ab_lib.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" 1 || exit 1
for w in "--scale 26" "--workload twitter" "--workload lj"; do
  n=$(echo $w | tr -d ' -')
  rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python bench.py $w --steps 2 --warmup 1 --no-cpu-baseline > $O/tr_$n.log 2>&1 || exit 1
  f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1); s=$(find $O/tr -name 'run_kernel_stats.csv' | head -1)
  python scripts/kb_timeline.py $f > $O/${n}_kb_timeline.txt; python scripts/step_gaps.py $f > $O/${n}_step_gaps.txt; cp $s $O/${n}_kernel_stats.csv
  rm -rf $O/tr
done
