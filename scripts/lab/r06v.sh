# Round 6 analysis (no product change): where the map's chunk time goes.  The lab library of
# scripts/lab/stamp_map.py (k_kb_map with clock stamps at four points of its chunk loop) in
# place of libsheep_amd.so; per-phase clocks for the non-hub (map) and hub (map_hub) variants
# over 3 RMAT-26 and 2 twitter-shape steps.
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
L=sheep_amd/libsheep_amd.so
cp $L $O/prod.so.tmp
cp sheep_amd/libsheep_amd_lab.so $L
timeout -k 10 300 python scripts/lab/stamps.py --steps 3 --names map map_hub > $O/stamps_r26.json 2> $O/stamps.err
r1=$?
timeout -k 10 300 python scripts/lab/stamps.py --workload twitter --steps 2 --names map map_hub > $O/stamps_twitter.json 2>> $O/stamps.err
r2=$?
cp $O/prod.so.tmp $L; rm -f $O/prod.so.tmp
[ $r1 -eq 0 ] && [ $r2 -eq 0 ] && cat $O/stamps_r26.json $O/stamps_twitter.json
