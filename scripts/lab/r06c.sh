# Round 6: the tile-mapped second partition pass (ff_groups 1, the new default) against the
# library at 304d53e (base: region search per tile, holes read and masked), alternating on one
# box; then kernel traces of RMAT-26, twitter and LJ at HEAD (kb timeline, step gaps, stats).
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
OUT=$O bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
for w in "--scale 26" "--workload twitter" "--workload lj"; do
  n=$(echo $w | tr -d ' -')
  rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python bench.py $w --steps 2 --warmup 1 --no-cpu-baseline > $O/tr_$n.log 2>&1 || exit 1
  f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1); s=$(find $O/tr -name 'run_kernel_stats.csv' | head -1)
  python scripts/kb_timeline.py $f > $O/${n}_kb_timeline.txt; python scripts/step_gaps.py $f > $O/${n}_step_gaps.txt; cp $s $O/${n}_kernel_stats.csv
  rm -rf $O/tr
done
