# Round 6: three builds alternating — base (sheep_amd/libsheep_amd_base.so, 476fcbf: before the
# spine ballots), spine (29c8be2: the spine's word searches as wave ballots), new (4f14bc0:
# + fresh maps on the applies' stream).  r06m mixed the two changes: RMAT-22 tree -0.06 ms,
# LJ +0.08 ms.  Small configs first (the kb loop's fixed costs matter most there).
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
L=sheep_amd/libsheep_amd.so
for r in 1 2 3; do
  for v in base spine new; do
    cp sheep_amd/libsheep_amd_$v.so $L
    for a in "--workload lj --steps 20 --warmup 3" "--scale 22 --seed 22 --steps 20 --warmup 3" "--steps 10 --warmup 3"; do
      line=$(timeout -k 10 240 python bench.py $a --no-cpu-baseline 2>>$O/ab.err) || { cp sheep_amd/libsheep_amd_new.so $L; exit 1; }
      echo "{\"lib\": \"$v\", \"args\": \"$a\", \"line\": $line}" >> $O/ab.jsonl
    done
    echo "round $r $v done"
  done
done
cp sheep_amd/libsheep_amd_new.so $L
