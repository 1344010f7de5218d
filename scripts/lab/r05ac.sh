# The pipelined kb timeline of the LJ shape at rank cuts 12 (the sweep's +2.5 ms cliff) and at
# the defaults.
export TMPDIR=/tmp
O=gpurun_out/r05ac; mkdir -p $O
for E in "SHEEP_KB_RANKB=12" "SHEEP_KB_RANKB=8"; do
  tag=$(echo $E | tr ' =' '__')
  rm -rf $O/tr && env $E SHEEP_KB_BUCKETS=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --workload lj --steps 3 --warmup 2 --no-cpu-baseline > $O/$tag.log 2>&1 || exit 1
  f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
  python scripts/kb_timeline.py $f > $O/lj_${tag}_kb_timeline.txt || exit 1
  rm -rf $O/tr
done
