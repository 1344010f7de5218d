# Round 6: hub-bucket maps with two 512-thread blocks per CU (k_kb_map KM2, kb_map2).
# Hypothesis: in the hub buckets the maps are the kb loop's critical path (RMAT-26 buckets
# 12-22, twitter 19-32: map 0.25-0.5 ms beside applies of 0.1-0.3 ms; profiles/r06/m_map2/
# timelines) and run at ~1.5 TB/s: one chunk in flight per CU, a chain of memory latencies per
# chunk.  Two blocks per CU overlap two chains.  The GPU suite first (full-size C2-C5 have hub
# buckets); then SHEEP_KB_MAP2=0/1 alternating, three rounds.
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
  for v in 0 1; do
    for a in "--steps 10 --warmup 3" "--workload twitter --steps 5 --warmup 2" "--scale 25 --seed 25 --steps 10 --warmup 3"; do
      line=$(SHEEP_KB_MAP2=$v timeout -k 10 240 python bench.py $a --no-cpu-baseline 2>>$O/ab.err) || exit 1
      echo "{\"v\": \"$v\", \"args\": \"$a\", \"line\": $line}" >> $O/ab.jsonl
    done
    echo "round $r map2=$v done"
  done
done
