# Round 6: the fused pass's cursors spread 512 B per line of 8 (SHEEP_FS_CLS 64, the new default)
# and the x-digit counts spread 512 B per line of 16 (xh_ix), against the contiguous layout (base
# = sheep_amd/libsheep_amd_base.so, HEAD d533cb9 built with SHEEP_FS_CLS=8).  r06h found the fused
# pass at 6.96 (cls 64) vs 7.56 (cls 8) vs 7.48 ms (cls 512, 4 KB apart) on one box, and the
# contiguous layout at 6.86 in the bench but 7.5 under rocprofv3 on another: the cursor atomics'
# speed depends on the memory channels their lines land on.  The GPU suite on new; bench lines
# alternating; rocprofv3 kernel stats of both (does the profiler still see another time?).
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 1 || exit 1
L=sheep_amd/libsheep_amd.so
cp $L $O/new.so.tmp
for v in new base; do
  if [ $v = base ]; then cp sheep_amd/libsheep_amd_base.so $L; else cp $O/new.so.tmp $L; fi
  rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/tr_$v.log 2>&1 || { cp $O/new.so.tmp $L; exit 1; }
  s=$(find $O/tr -name 'run_kernel_stats.csv' | head -1); cp $s $O/${v}_kernel_stats.csv; rm -rf $O/tr
done
cp $O/new.so.tmp $L; rm -f $O/new.so.tmp
