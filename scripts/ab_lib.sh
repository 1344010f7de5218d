#!/bin/bash
# A/B of two builds of the library on one box: sheep_amd/libsheep_amd.so (new) against
# sheep_amd/libsheep_amd_base.so (base), alternating, one bench process per run.
#   OUT=gpurun_out/ablib bash scripts/ab_lib.sh "<bench args>" [rounds]
set -o pipefail
OUT=${OUT:-gpurun_out/ablib}
mkdir -p "$OUT"
ARGS=$1
N=${2:-2}
L=sheep_amd/libsheep_amd.so
cp "$L" "$OUT/new.so.tmp" || exit 1
for i in $(seq 1 "$N"); do
  for v in base new; do
    if [ $v = base ]; then cp sheep_amd/libsheep_amd_base.so "$L"; else cp "$OUT/new.so.tmp" "$L"; fi
    line=$(timeout -k 10 240 python bench.py $ARGS 2>> "$OUT/ab.err") || { cp "$OUT/new.so.tmp" "$L"; echo "run failed: $v"; exit 1; }
    python - "$v" "$ARGS" "$line" >> "$OUT/ab.jsonl" <<'PY'
import json, sys
r = json.loads(sys.argv[3])
ph = (r.get("roofline") or {}).get("phases_ms", {})
print(json.dumps({"lib": sys.argv[1], "args": sys.argv[2], "ms": round(r["ms_per_step"], 3), "phases": ph}))
PY
    echo "done: $v"
  done
done
cp "$OUT/new.so.tmp" "$L"
rm -f "$OUT/new.so.tmp"
