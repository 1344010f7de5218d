# HEAD: the P = 8 lockstep simulation (per-rank front half measured), the multi-rank driver as a
# one-rank RCCL group against the single path, and RMAT-22 / LJ per-bucket zipper stats.
export TMPDIR=/tmp
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 300 python scripts/lockstep_sim.py --P 8 --reps 2 > $O/sim.jsonl 2>$O/sim.err || exit 1
echo sim ok
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/single_$i.json 2>>$O/bench.err || exit 1
  timeout -k 10 240 python bench.py --lockstep-1 --no-cpu-baseline --steps 10 --warmup 3 > $O/lockstep1_$i.json 2>>$O/bench.err || exit 1
done
echo lockstep ok
SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --scale 22 --seed 22 --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> $O/r22_per_bucket.txt || exit 1
SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --workload lj --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> $O/lj_per_bucket.txt || exit 1
