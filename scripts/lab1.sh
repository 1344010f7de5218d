set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export LAB_STATS=0
SHEEP_KB_RANKB=64 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof2 -o run -- python scripts/tree_lab.py --scale 26 --reps 1 --variants kb:64 > gpurun_out/prof2.log 2>&1 &&
SCALE=26 timeout -k 10 300 bash scripts/lab_env.sh "SHEEP_KB_MAPMODE=3:kb:64" "SHEEP_KB_MAPMODE=0:kb:64" "SHEEP_KB_MAPMODE=0,SHEEP_KB_RANKB=64:kb:64" "SHEEP_KB_MAPMODE=0,SHEEP_KB_RANKB=16:kb:64" "SHEEP_KB_MAPMODE=0,SHEEP_KB_RANKB=64:kb:32"  > gpurun_out/lab_mm.log 2>&1
