# Round 6, final check of the in-tree library at HEAD (the one the round-end driver loads): the
# GPU suite, smoke() and the default bench line.
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py > $O/bench_rmat26.json 2> $O/bench.err && echo "bench ok" && cat $O/bench_rmat26.json
