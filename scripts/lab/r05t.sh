# (round 6) Added with its results in commit 99fef59: SHEEP_LAB 8 (histogram rounds with the next loads in flight) was built in the gitignored csrc_lab copy; adopted. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# A/B: SHEEP_LAB=8 = k_degb_hist16s in rounds of 65528 entries with the next round's first
# half loaded during the fold, the fold clearing the counters (no zeroing pass).
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
SHEEP_LAB=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py tests/test_multi_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_lab8.log 2>&1 || { tail -30 $O/pytest_lab8.log; exit 1; }
tail -2 $O/pytest_lab8.log
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=8 - SHEEP_LAB=8 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=8 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --check --steps 2 --warmup 1" SHEEP_LAB=8 || exit 1
# the RMAT-26 kb timeline and step gaps at this build (default settings)
rm -rf $O/tr_r26 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_r26 -o run -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/r26.log 2>&1 || exit 1
f=$(find $O/tr_r26 -name 'run_kernel_trace.csv' | head -1)
python scripts/kb_timeline.py $f > $O/r26_kb_timeline.txt || exit 1
python scripts/step_gaps.py $f > $O/r26_gaps.txt || exit 1
cp $(find $O/tr_r26 -name 'run_kernel_stats.csv' | head -1) $O/r26_kernel_stats.csv
rm -rf $O/tr_r26
