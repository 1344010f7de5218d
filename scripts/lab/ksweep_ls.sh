# lockstep P=8 simulation: bucket count sweep (apply is the serial part)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ksweep_ls.log
for K in 40 48 56 64; do SHEEP_KB_BUCKETS=$K SHEEP_KB_RANKB=$K timeout -k 10 300 python scripts/lockstep_sim.py --scale 26 --P 8 --reps 2 >> gpurun_out/ksweep_ls.log 2>&1 || exit 1; echo "K=$K ok"; done
