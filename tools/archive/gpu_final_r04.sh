#!/bin/bash
# Round-4 closing check on the final tree: smoke(), the multi-rank test, the default bench line.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/r04w
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_multirank.py > $OUT/multirank.log 2>&1 || { echo "multirank failed"; tail -5 $OUT/multirank.log; exit 1; }
tail -2 $OUT/multirank.log
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2> $OUT/bench_default.err || { echo "bench rc=$?"; tail -5 $OUT/bench_default.err; exit 1; }
cut -c1-300 $OUT/bench_default.log
cat $OUT/bench_default.err | grep "^\[bench"
