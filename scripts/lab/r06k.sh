# Round 6 sweep: the default bucket rules across R-MAT scales 21-25 x 3
# seeds, LJ and twitter; at scales 22 / 23 (the only ones inside the dense-cut class, 1.5 x 2^25
# .. 1.5 x 2^27 records with mean degree >= 40) also with the rule off (SHEEP_KB_RANKB = the
# automatic count: 8 / 16).  Two alternating runs per setting.
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
for s in 21 22 23 24 25; do
  st=20; [ $s -ge 24 ] && st=10
  for seed in $s 3 7; do
    E="-"
    [ $s = 22 ] && E="SHEEP_KB_RANKB=8"
    [ $s = 23 ] && E="SHEEP_KB_RANKB=16"
    if [ "$E" = "-" ]; then
      OUT=$O bash scripts/ab_env.sh "--scale $s --seed $seed --no-cpu-baseline --steps $st --warmup 3" - - || exit 1
    else
      OUT=$O bash scripts/ab_env.sh "--scale $s --seed $seed --no-cpu-baseline --steps $st --warmup 3" - $E - $E || exit 1
    fi
  done
done
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" - - || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - - || exit 1
