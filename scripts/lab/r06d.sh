# Round 6: the refresh makes the zipper's first step of the pairs from pre-bucket roots
# (SHEEP_KB_RLINK=1, new default): the GPU suite, then bench lines alternating 1 / 0, and the
# RMAT-26 kb timeline at 1.
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_KB_RLINK=0 - SHEEP_KB_RLINK=0 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_KB_RLINK=0 - SHEEP_KB_RLINK=0 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_KB_RLINK=0 - SHEEP_KB_RLINK=0 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_KB_RLINK=0 || exit 1
rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/tr.log 2>&1 || exit 1
f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
python scripts/kb_timeline.py $f > $O/r26_kb_timeline.txt; rm -rf $O/tr
