# Birth-window width sweep (SHEEP_KB_FRESH_LO / _HI, hundredths of the mean degree): does a
# wider window of fresh (unpipelined) buckets remove the small configs' cliffs, and at what cost?
export TMPDIR=/tmp
O=gpurun_out/r05ae; mkdir -p $O
W1="SHEEP_KB_FRESH_LO=40 SHEEP_KB_FRESH_HI=150"
W2="SHEEP_KB_FRESH_LO=30 SHEEP_KB_FRESH_HI=200"
W3="SHEEP_KB_FRESH_LO=50 SHEEP_KB_FRESH_HI=200"
for a in "--scale 22 --seed 22" "--scale 22 --seed 5" "--scale 22 --seed 9" "--workload lj" "--scale 23 --seed 23" "--scale 24 --seed 24"; do
  OUT=$O bash scripts/ab_env.sh "$a --no-cpu-baseline --steps 20 --warmup 3" - "$W1" "$W2" "$W3" "$W2 SHEEP_KB_RANKB=12" || exit 1
done
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - "$W1" "$W2" "$W3" || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 26 --seed 5 --no-cpu-baseline --steps 6 --warmup 2" - "$W1" "$W2" "$W3" || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - "$W1" "$W2" "$W3" || exit 1
