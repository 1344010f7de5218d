# A/B (base = HEAD 99fef59, new = k_degb_hist with dynamic LDS (two blocks per CU for small
# buckets) and double-buffered loads), small configs; the GPU suite on new; the RMAT-26 kb
# timeline and gaps at new.
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --no-cpu-baseline --steps 20 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 3 || exit 1
rm -rf $O/tr_r26 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_r26 -o run -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/r26.log 2>&1 || exit 1
f=$(find $O/tr_r26 -name 'run_kernel_trace.csv' | head -1)
python scripts/kb_timeline.py $f > $O/r26_kb_timeline.txt || exit 1
python scripts/step_gaps.py $f > $O/r26_gaps.txt || exit 1
cp $(find $O/tr_r26 -name 'run_kernel_stats.csv' | head -1) $O/r26_kernel_stats.csv
rm -rf $O/tr_r26
