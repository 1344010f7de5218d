# Round 6 lab: the fused pass's region cursors spread over memory (SHEEP_FS_CLS: u64 between
# consecutive 64-B lines of 8 cursors; 8 = contiguous, the build before).  Hypothesis: the
# ~134 M cursor atomics per call are performed at the memory side, and 2 x 8 KB of contiguous
# cursors sit on a few HBM channels, so the fused pass's time depends on where the allocator
# put them (bench 6.86 ms vs 7.49-7.62 ms under rocprofv3 in one lease, profiles/r06/ev/).
# Builds: sheep_amd/libsheep_amd_cls{8,64,512}.so (hipcc -DSHEEP_FS_CLS=N, untracked).
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
L=sheep_amd/libsheep_amd.so
cp $L $O/head.so.tmp || exit 1
for N in 512 64; do
  cp sheep_amd/libsheep_amd_cls$N.so $L
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sampled or fused or fullsize_tree" > $O/pytest_cls$N.log 2>&1; rc=$?; tail -1 $O/pytest_cls$N.log; [ $rc = 0 ] || { cp $O/head.so.tmp $L; exit 1; }
done
for r in 1 2; do
  for N in 8 64 512; do
    cp sheep_amd/libsheep_amd_cls$N.so $L
    line=$(timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --warmup 3 2>>$O/ab.err) || { cp $O/head.so.tmp $L; exit 1; }
    echo "{\"cls\": $N, \"line\": $line}" >> $O/ab_rmat26.jsonl
    line=$(timeout -k 10 240 python bench.py --workload twitter --no-cpu-baseline --steps 6 --warmup 2 2>>$O/ab.err) || { cp $O/head.so.tmp $L; exit 1; }
    echo "{\"cls\": $N, \"line\": $line}" >> $O/ab_twitter.jsonl
    echo "round $r cls $N done"
  done
done
for N in 8 512; do
  cp sheep_amd/libsheep_amd_cls$N.so $L
  rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/tr_cls$N.log 2>&1 || { cp $O/head.so.tmp $L; exit 1; }
  s=$(find $O/tr -name 'run_kernel_stats.csv' | head -1); cp $s $O/cls${N}_kernel_stats.csv; rm -rf $O/tr
done
cp $O/head.so.tmp $L; rm -f $O/head.so.tmp
