# Round 6: star paths in the birth window's buckets (k_kb_star_path, kb_star).  Hypothesis: the
# percolation bucket's long zipper walks (LJ shape: 250 K of its 441 K zipped pairs start at a
# pre-bucket root the refresh could not link, max walk ~900 steps; profiles/r06/j_pick2/) are
# stars — many pairs of one root, each walking up the root's growing chain; as the path over
# their sorted ends they take about one step each, for a sort of the bucket's star keys.
# The GPU suite at the new default first; then per-bucket zipper stats of LJ / RMAT-22 under
# both builds (SHEEP_TREE_STATS=2: unpipelined); then three alternating rounds of bench lines.
# base = libsheep_amd_base.so (e0a7e8e), star = libsheep_amd_star.so.
export TMPDIR=/tmp
O=gpurun_out/r06q; mkdir -p $O
L=sheep_amd/libsheep_amd.so
cp sheep_amd/libsheep_amd_star.so $L
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in base star; do
  cp sheep_amd/libsheep_amd_$v.so $L
  SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --workload lj --steps 1 --warmup 0 --no-cpu-baseline > $O/stats_lj_$v.json 2> $O/stats_lj_$v.txt || { cp sheep_amd/libsheep_amd_star.so $L; exit 1; }
  SHEEP_TREE_STATS=2 timeout -k 10 240 python bench.py --scale 22 --seed 22 --steps 1 --warmup 0 --no-cpu-baseline > $O/stats_r22_$v.json 2> $O/stats_r22_$v.txt || { cp sheep_amd/libsheep_amd_star.so $L; exit 1; }
done
echo "stats done"
for r in 1 2 3; do
  for v in base star; do
    cp sheep_amd/libsheep_amd_$v.so $L
    for a in "--workload lj --steps 20 --warmup 3" "--scale 22 --seed 22 --steps 20 --warmup 3" "--workload twitter --steps 5 --warmup 2" "--steps 10 --warmup 3"; do
      line=$(timeout -k 10 240 python bench.py $a --no-cpu-baseline 2>>$O/ab.err) || { cp sheep_amd/libsheep_amd_star.so $L; exit 1; }
      echo "{\"lib\": \"$v\", \"args\": \"$a\", \"line\": $line}" >> $O/ab.jsonl
    done
    echo "round $r $v done"
  done
done
cp sheep_amd/libsheep_amd_star.so $L
