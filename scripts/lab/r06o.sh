# Round 6: the split apply's bucket owners.  Hypothesis: round-robin
# (k mod P) leaves the per-rank applies 3.7-4.8 ms apart at P = 8 because the owners' refreshes
# of all P x cap pairs land unevenly; owners chosen by the fewest owned pairs so far should cut
# max / min apply towards 1.15 and the simulated critical path by ~0.5 ms.  SHEEP_LS_OWNER 0 / 1
# alternating, P = 8 lockstep simulation at RMAT-26 (bit-exact check inside), then the
# multi-rank parity tests at the new default.
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    SHEEP_LS_OWNER=$v timeout -k 10 300 python scripts/lockstep_sim.py --P 8 --reps 2 > $O/sim_owner${v}_$r.jsonl 2>> $O/sim.err || exit 1
    echo "round $r owner $v done"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_multi_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_multi.log 2>&1 && tail -1 $O/pytest_multi.log
