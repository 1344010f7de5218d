# (round 6) SHEEP_KB_ZGRID was a lab knob, removed after this run (rejected: DESIGN §9).
# Round 6 lab: the zipper's grid (SHEEP_KB_ZGRID, lab knob; default 2048 blocks = every chunk of
# the kept pairs in flight at once).  Hypothesis: the percolation bucket's one long insertion
# (LJ ~900 steps, 1.15 ms) comes from inserting the bucket's pairs all at once, out of rank
# order; a narrower window (fewer blocks sweeping the pairs in increasing order) would shorten
# it.  LJ and RMAT-22 kb timelines at 2048 / 256 / 64 blocks, and bench lines.
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_KB_ZGRID=256 SHEEP_KB_ZGRID=64 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_KB_ZGRID=256 SHEEP_KB_ZGRID=64 || exit 1
for z in 2048 256 64; do
  rm -rf $O/tr && SHEEP_KB_ZGRID=$z timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --workload lj --steps 2 --warmup 1 --no-cpu-baseline > $O/tr_$z.log 2>&1 || exit 1
  f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
  python scripts/kb_timeline.py $f > $O/lj_z${z}_kb_timeline.txt; rm -rf $O/tr
done
