# rocprofv3 kernel stats of the one-GPU lockstep simulation (P shards of RMAT-26)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_sim
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sim -o run -- python scripts/lockstep_sim.py --scale 26 --P ${P:-8} --reps 1 > gpurun_out/prof_sim.log 2>&1 && echo "prof ok"
