# Round 6: the anchor pick's dominance threshold.  Hypothesis: the percolation bucket's long
# zipper walk (LJ ~900 steps, ~1 ms of a 3.2 ms tree) is the star of the largest pre-bucket
# component: its pairs all start at one etree root and walk its growing chain.  With the
# anchor on that component (the pick taking the component with the most samples from 2 of 256
# instead of 3), its pairs become marks and the spine builds its chain in rank order.
# base = libsheep_amd_base.so (e0a7e8e), pick2 = libsheep_amd_pick2.so.  First the per-bucket
# zipper stats of the LJ shape under both (SHEEP_TREE_STATS=2: unpipelined), then three
# alternating rounds of bench lines.
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
L=sheep_amd/libsheep_amd.so
cp $L $O/cur.so.tmp
for v in base pick2; do
  cp sheep_amd/libsheep_amd_$v.so $L
  SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --workload lj --steps 1 --warmup 0 --no-cpu-baseline > $O/stats_lj_$v.json 2> $O/stats_lj_$v.txt || { cp $O/cur.so.tmp $L; exit 1; }
  SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --scale 22 --seed 22 --steps 1 --warmup 0 --no-cpu-baseline > $O/stats_r22_$v.json 2> $O/stats_r22_$v.txt || { cp $O/cur.so.tmp $L; exit 1; }
done
echo "stats done"
for r in 1 2 3; do
  for v in base pick2; do
    cp sheep_amd/libsheep_amd_$v.so $L
    for a in "--workload lj --steps 20 --warmup 3" "--scale 22 --seed 22 --steps 20 --warmup 3" "--workload twitter --steps 5 --warmup 2" "--steps 10 --warmup 3"; do
      line=$(timeout -k 10 240 python bench.py $a --no-cpu-baseline 2>>$O/ab.err) || { cp $O/cur.so.tmp $L; exit 1; }
      echo "{\"lib\": \"$v\", \"args\": \"$a\", \"line\": $line}" >> $O/ab.jsonl
    done
    echo "round $r $v done"
  done
done
cp $O/cur.so.tmp $L; rm -f $O/cur.so.tmp
