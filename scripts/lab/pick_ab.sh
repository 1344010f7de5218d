set -o pipefail
export TMPDIR=/tmp
bash scripts/ab_knob.sh '{}' '{"kb_pick": 0}' '{}' &&
timeout -k 10 300 python scripts/map_lab.py --workload twitter --reps 2 '{}' '{"kb_pick": 0}' '{"kb_buckets": 40, "kb_rankb": 40}' '{"kb_buckets": 40, "kb_rankb": 40, "kb_pick": 0}' > gpurun_out/pick_tw.log 2>&1 &&
timeout -k 10 300 python scripts/map_lab.py --scale 22 --reps 5 '{}' '{"kb_pick": 0}' > gpurun_out/pick_22.log 2>&1 &&
grep -h '^{' gpurun_out/pick_tw.log gpurun_out/pick_22.log | cut -c1-420
