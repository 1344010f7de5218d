# Round 6: memory placement of the front half's atomic counters.  Three builds, alternating:
#   base: libsheep_amd_base.so = HEAD d533cb9 built with SHEEP_FS_CLS=8: the fused pass's 2 x 1024
#         region cursors contiguous (8 KB each), the x-digit counts contiguous (1 KB);
#   new:  libsheep_amd_new.so  = the cursors 512 B per line of 8 (SHEEP_FS_CLS 64), the x-digit
#         counts 512 B per line of 16 (xh_ix) — the default build;
#   xc:   libsheep_amd_xc.so   = new + the second pass's 256 x-digit cursors spread as well.
# r06h found the fused pass at 6.96 (spread 512 B) vs 7.56 (contiguous) vs 7.48 ms (4 KB apart)
# on one box, and the contiguous layout at 6.86 ms in a bench line but 7.5 ms under rocprofv3
# on another: the atomics' speed depends on the memory channels their lines land on.
# The GPU suite on new, a parity subset on xc, bench lines, rocprofv3 kernel stats of each.
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
L=sheep_amd/libsheep_amd.so
cp sheep_amd/libsheep_amd_new.so $L
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
cp sheep_amd/libsheep_amd_xc.so $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sampled or fused or fullsize_tree or front_half" > $O/pytest_xc.log 2>&1; rc=$?; tail -1 $O/pytest_xc.log; [ $rc = 0 ] || { cp sheep_amd/libsheep_amd_new.so $L; exit 1; }
for r in 1 2; do
  for v in base new xc; do
    cp sheep_amd/libsheep_amd_$v.so $L
    line=$(timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --warmup 3 2>>$O/ab.err) || { cp sheep_amd/libsheep_amd_new.so $L; exit 1; }
    echo "{\"lib\": \"$v\", \"line\": $line}" >> $O/ab_rmat26.jsonl
    line=$(timeout -k 10 240 python bench.py --workload twitter --no-cpu-baseline --steps 6 --warmup 2 2>>$O/ab.err) || { cp sheep_amd/libsheep_amd_new.so $L; exit 1; }
    echo "{\"lib\": \"$v\", \"line\": $line}" >> $O/ab_twitter.jsonl
    echo "round $r $v done"
  done
done
for v in base new xc; do
  cp sheep_amd/libsheep_amd_$v.so $L
  rm -rf $O/tr && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/tr_$v.log 2>&1 || { cp sheep_amd/libsheep_amd_new.so $L; exit 1; }
  s=$(find $O/tr -name 'run_kernel_stats.csv' | head -1); cp $s $O/${v}_kernel_stats.csv; rm -rf $O/tr
done
cp sheep_amd/libsheep_amd_new.so $L
