# Kernel traces of the small configs at HEAD (LJ, RMAT-22): kb timeline, step gaps, kernel stats.
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
for c in "lj:--workload lj" "r22:--scale 22 --seed 22" "r26:--scale 26"; do
  n=${c%%:*}; a=${c#*:}
  rm -rf $O/tr_$n && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$n -o run -- python bench.py $a --steps 3 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || exit 1
  f=$(find $O/tr_$n -name 'run_kernel_trace.csv' | head -1)
  s=$(find $O/tr_$n -name 'run_kernel_stats.csv' | head -1)
  python scripts/kb_timeline.py $f > $O/${n}_kb_timeline.txt || exit 1
  python scripts/step_gaps.py $f > $O/${n}_gaps.txt || exit 1
  cp $s $O/${n}_kernel_stats.csv
  rm -rf $O/tr_$n
done
