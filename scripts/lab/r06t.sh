# Round 6: the split apply in a group of one.  Hypothesis: with the zipper of each bucket on its
# own stream (the split apply's forest part) and the union-find part computed from the pairs,
# the percolation bucket's long zipper (twitter 2.3 ms, LJ ~1 ms, RMAT-26 ~1 ms per tree) leaves
# the applies' critical path.  bench.py --lockstep-1 (the multi-rank driver over a one-rank RCCL
# group) with SHEEP_LS_SPLIT=2 (split at P = 1) against the default lockstep-1 and the single
# path, alternating, three rounds.
export TMPDIR=/tmp
O=gpurun_out/r06t; mkdir -p $O
for r in 1 2 3; do
  for a in "--workload lj --steps 20 --warmup 3" "--workload twitter --steps 5 --warmup 2" "--steps 10 --warmup 3" "--scale 22 --seed 22 --steps 20 --warmup 3"; do
    for v in single ls1 ls1split; do
      case $v in
        single) line=$(timeout -k 10 240 python bench.py $a --no-cpu-baseline 2>>$O/ab.err) ;;
        ls1) line=$(timeout -k 10 240 python bench.py $a --lockstep-1 --no-cpu-baseline 2>>$O/ab.err) ;;
        ls1split) line=$(SHEEP_LS_SPLIT=2 timeout -k 10 240 python bench.py $a --lockstep-1 --no-cpu-baseline 2>>$O/ab.err) ;;
      esac
      [ -n "$line" ] || exit 1
      echo "{\"v\": \"$v\", \"args\": \"$a\", \"line\": $line}" >> $O/ab.jsonl
    done
  done
  echo "round $r done"
done
