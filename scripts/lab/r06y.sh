# Round 6, second form: the window's END from the device signal (fresh from
# the mean degree crossing kb_fresh_lo until the pick has seen a dominant component). First form
# (r06x: fresh from the first bucket) in profiles/r06/o_birth_signal/ab_first.jsonl.
# Before: the kb loop's fresh maps from a device-side birth signal
# (kb_birth: every map fresh until the pick before it has seen a dominant component, >= 3 of
# 256 samples; the giant sweeps start once the host has read that flag) instead of the
# mean-degree window 0.5-1.0 (kb_fresh_lo / _hi).  Parity first with kb_birth on (the tree
# tests and the full-size digests), then the item-3 sweep: R-MAT 21-25 x 3 seeds, LJ, twitter,
# default / SHEEP_KB_BIRTH=1 alternating, two rounds each.
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
SHEEP_KB_BIRTH=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py tests/test_multi_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_birth.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_birth.log; exit 1; }
tail -1 $O/pytest_birth.log
for s in 21 22 23 24 25; do
  st=12; [ $s -ge 24 ] && st=8
  for seed in $s 3 7; do
    OUT=$O bash scripts/ab_env.sh "--scale $s --seed $seed --no-cpu-baseline --steps $st --warmup 2" - SHEEP_KB_BIRTH=1 - SHEEP_KB_BIRTH=1 || exit 1
  done
done
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 12 --warmup 2" - SHEEP_KB_BIRTH=1 - SHEEP_KB_BIRTH=1 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 5 --warmup 2" - SHEEP_KB_BIRTH=1 - SHEEP_KB_BIRTH=1 || exit 1
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 8 --warmup 2" - SHEEP_KB_BIRTH=1 - SHEEP_KB_BIRTH=1 || exit 1
