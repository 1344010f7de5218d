# (round 6) Added with its results in commit cb15880: SHEEP_LAB 16 / 32 (fused-pass grid and write order) were built in the gitignored csrc_lab copy; measurement only, neither adopted. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# Fused pass: WRITE_SIZE and time with the persistent grid (default) and one block per tile
# (SHEEP_LAB=16) and y runs written before x runs (SHEEP_LAB=32)
export TMPDIR=/tmp
O=gpurun_out/r05y2; mkdir -p $O
for E in "-" "SHEEP_LAB=32"; do
  n=$([ "$E" = "-" ] && echo base || echo lab32)
  EE=$([ "$E" = "-" ] && echo "" || echo "$E")
  rm -rf $O/w_$n && env $EE timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/w_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
  python scripts/lab/kernel_pmc.py $O/w_$n WRITE_SIZE > $O/w_$n.txt && cat $O/w_$n.txt
  rm -rf $O/w_$n
done
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=32 - SHEEP_LAB=32 || exit 1
