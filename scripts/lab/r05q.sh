# (round 6) Added with its results in commit 5b56007: SHEEP_LAB bits 1 / 2 (persistent fused pass, Eytzinger bin search) were built in the gitignored csrc_lab copy; both adopted. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# Lab A/B: SHEEP_LAB bit 1 = persistent fused front pass with the next tile's records loaded
# under the y write-out; bit 2 = k_edge_bin's bin search over an Eytzinger-ordered table.
# The GPU suite runs once with both on, then bench lines alternate the settings.
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
SHEEP_LAB=3 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_lab3.log 2>&1 || { tail -30 $O/pytest_lab3.log; exit 1; }
tail -2 $O/pytest_lab3.log
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=1 SHEEP_LAB=2 SHEEP_LAB=3 - SHEEP_LAB=1 SHEEP_LAB=2 SHEEP_LAB=3 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=3 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --no-cpu-baseline --check --steps 20 --warmup 3" - SHEEP_LAB=3 || exit 1
