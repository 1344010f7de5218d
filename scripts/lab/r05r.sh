# A/B: timing events pooled in the context (new) vs created/destroyed per call (base, HEAD
# 5b56007); then kernel traces of the small configs with the new library (kb timeline, gaps).
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --no-cpu-baseline --steps 20 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 2 || exit 1
for c in "lj:--workload lj" "r22:--scale 22 --seed 22"; do
  n=${c%%:*}; a=${c#*:}
  rm -rf $O/tr_$n && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$n -o run -- python bench.py $a --steps 3 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || exit 1
  f=$(find $O/tr_$n -name 'run_kernel_trace.csv' | head -1)
  python scripts/kb_timeline.py $f > $O/${n}_kb_timeline.txt || exit 1
  python scripts/step_gaps.py $f --min-us 5 > $O/${n}_gaps.txt || exit 1
  cp $f $O/${n}_trace.csv
  rm -rf $O/tr_$n
done
