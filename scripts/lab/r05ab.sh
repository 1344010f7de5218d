# Per-bucket zipper stats (SHEEP_TREE_STATS=2) of the small configs at rank cuts 12 + edge cuts
# 8 (the sweep's cliff on LJ, the gain on RMAT-22) and at the defaults, with tree times.
export TMPDIR=/tmp
O=gpurun_out/r05ab; mkdir -p $O
for E in "SHEEP_KB_RANKB=12 SHEEP_KB_BUCKETS=8" "SHEEP_KB_RANKB=8 SHEEP_KB_BUCKETS=8"; do
  tag=$(echo $E | tr ' =' '__')
  env $E SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --workload lj --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> $O/lj_$tag.txt || exit 1
  env $E SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --scale 22 --seed 22 --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> $O/r22_$tag.txt || exit 1
done
