# (round 6) Added with its results in commit df0b782: the birth-window split (SHEEP_LAB_BIRTH_SPLIT) was built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_BIRTH_SPLIT=2 SHEEP_LAB_BIRTH_SPLIT=4 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_BIRTH_SPLIT=2 SHEEP_LAB_BIRTH_SPLIT=4 || exit 1
OUT=$O bash scripts/ab_env.sh "--steps 8 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_BIRTH_SPLIT=2 SHEEP_LAB_BIRTH_SPLIT=4 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_BIRTH_SPLIT=2 SHEEP_LAB_BIRTH_SPLIT=4 || exit 1
rm -rf $O/tr && SHEEP_KB_PIPE=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/tr.log 2>&1 || exit 1
f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
python scripts/kb_timeline.py $f > $O/r26_kb_timeline_nopipe.txt
rm -rf $O/tr
