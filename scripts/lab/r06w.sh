# Round 6: the map's per-chunk wave offsets as a shuffle scan in wave 0 instead of thread 0's
# 16 dependent LDS steps (the chunk's reservation phase: 27 % of the hub map's chunk,
# profiles/r06/n_map_stamps/), every other wave waiting at the barrier meanwhile.
# The GPU suite at the new build; then base (libsheep_amd_base.so, e0a7e8e) / scan alternating,
# three rounds.
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
L=sheep_amd/libsheep_amd.so
cp sheep_amd/libsheep_amd_scan.so $L
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
  for v in base scan; do
    cp sheep_amd/libsheep_amd_$v.so $L
    for a in "--steps 10 --warmup 3" "--workload twitter --steps 5 --warmup 2" "--workload lj --steps 20 --warmup 3" "--scale 22 --seed 22 --steps 20 --warmup 3"; do
      line=$(timeout -k 10 240 python bench.py $a --no-cpu-baseline 2>>$O/ab.err) || { cp sheep_amd/libsheep_amd_scan.so $L; exit 1; }
      echo "{\"v\": \"$v\", \"args\": \"$a\", \"line\": $line}" >> $O/ab.jsonl
    done
    echo "round $r $v done"
  done
done
cp sheep_amd/libsheep_amd_scan.so $L
