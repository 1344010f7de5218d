export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 300 python scripts/lockstep_sim.py --P 8 --reps 2 > $O/sim.jsonl 2>$O/sim.err || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_rmat26.json 2>$O/bench.err || exit 1
timeout -k 10 240 python bench.py --workload twitter --no-cpu-baseline --steps 6 --warmup 2 > $O/bench_twitter.json 2>>$O/bench.err || exit 1
timeout -k 10 240 python bench.py --workload lj --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_lj.json 2>>$O/bench.err || exit 1
timeout -k 10 240 python bench.py --scale 22 --seed 22 --check --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_rmat22_checked.json 2>>$O/bench.err || exit 1
SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> $O/r26_per_bucket.txt || exit 1
rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/tr.log 2>&1 || exit 1
f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
python scripts/kb_timeline.py $f > $O/r26_kb_timeline.txt; python scripts/step_gaps.py $f > $O/r26_step_gaps.txt
rm -rf $O/tr
