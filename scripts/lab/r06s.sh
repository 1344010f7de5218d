# Round 6: HIP API trace beside the kernel trace of the RMAT-22 and LJ lines, for the host time
# between two graph2tree calls (~180-220 us of idle device per step, scripts/step_gaps.py --prev)
# and the readback waits inside one.
export TMPDIR=/tmp
O=gpurun_out/r06s; mkdir -p $O
for w in "r22:--scale 22 --seed 22" "lj:--workload lj"; do
  n=${w%%:*}; a=${w#*:}
  rm -rf $O/$n
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/$n -o run -- python bench.py $a --steps 3 --warmup 1 --no-cpu-baseline > $O/$n.log 2>&1 || exit 1
  echo "$n ok"
done
