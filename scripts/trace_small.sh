#!/bin/bash
# Per-bucket tree kernel traces of the small configs (LJ shape, RMAT-22).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
WL=lj bash scripts/trace_tree.sh > /dev/null && cp gpurun_out/trace_buckets.txt gpurun_out/trace_buckets_lj.txt &&
cp gpurun_out/trace/run_kernel_trace.csv gpurun_out/trace_lj.csv &&
SCALE=22 bash scripts/trace_tree.sh > /dev/null && cp gpurun_out/trace_buckets.txt gpurun_out/trace_buckets_rmat22.txt &&
cp gpurun_out/trace/run_kernel_trace.csv gpurun_out/trace_rmat22.csv && tail -1 gpurun_out/trace_buckets_lj.txt && tail -1 gpurun_out/trace_buckets_rmat22.txt
