export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python scripts/lockstep_sim.py --P 8 --reps 2 > $O/sim_new.jsonl 2>$O/sim.err || exit 1
cp sheep_amd/libsheep_amd.so $O/new.so.tmp && cp sheep_amd/libsheep_amd_base.so sheep_amd/libsheep_amd.so
timeout -k 10 300 python scripts/lockstep_sim.py --P 8 --reps 2 > $O/sim_base.jsonl 2>>$O/sim.err; rc=$?
cp $O/new.so.tmp sheep_amd/libsheep_amd.so; rm -f $O/new.so.tmp; exit $rc
rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/tr.log 2>&1 || exit 1
f=$(ls $O/tr/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/tr/run_kernel_trace.csv)
python scripts/kb_timeline.py $f > $O/r26_kb_timeline.txt && python scripts/step_gaps.py $f > $O/r26_step_gaps.txt
rm -rf $O/tr
