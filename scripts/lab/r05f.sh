# (round 6) Added with its results in commit 173f10d: the giant-sweep schedules (SHEEP_LAB_SWEEP*) were built in the gitignored csrc_lab copy; adopted as the sweeps on the applies' stream (sweep_plan). The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
OUT=$O bash scripts/ab_env.sh "--steps 8 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=1 SHEEP_LAB_SWEEP=2 SHEEP_LAB_SWEEP=3 SHEEP_LAB_SWEEP=4 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=1 SHEEP_LAB_SWEEP=2 SHEEP_LAB_SWEEP=3 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=1 SHEEP_LAB_SWEEP=2 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=1 SHEEP_LAB_SWEEP=2 || exit 1
cp sheep_amd/libsheep_amd_lab.so sheep_amd/libsheep_amd.so
for w in "--scale 26" "--workload twitter" "--scale 22"; do timeout -k 10 200 python scripts/lab/stamps.py $w --steps 1 --raw >> $O/refresh.jsonl 2>>$O/err.log || exit 1; done
