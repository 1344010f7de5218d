# kernel trace of the lockstep loop over a one-rank RCCL group (host gaps between buckets)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ls1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ls1 -o run -- python bench.py --lockstep-1 --scale ${SCALE:-26} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ls1.log 2>&1 && echo "prof ok"
