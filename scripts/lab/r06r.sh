# Round 6: kernel traces of the twitter, LJ and RMAT-26 lines at HEAD, for the per-bucket
# timelines of the tree (scripts/kb_timeline.py) and the step gaps (scripts/step_gaps.py).
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
for w in "twitter:--workload twitter" "lj:--workload lj" "r26:"; do
  n=${w%%:*}; a=${w#*:}
  rm -rf $O/$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python bench.py $a --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.log 2>&1 || exit 1
  echo "$n ok"
done
