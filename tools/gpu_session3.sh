#!/bin/bash
# GPU session: full GPU test suite, smoke, default bench, then the north-star stand-in and the C5
# stand-in (environment light + Russian roulette). Stops at the first crash / timeout.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n ${TAIL:-6} "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py --steps 5 --warmup 1
step bench_ns 600 python bench.py --scene scenes/CBlucy_standin.dae --width 1920 --height 1080 --spp 128 --max-depth 5 --steps 3 --warmup 1 --no-cpu-baseline
step bench_c5 600 python bench.py --scene scenes/CBlucy_standin.dae --width 1920 --height 1080 --spp 128 --max-depth 8 --envmap synth:1024x512 --rr --steps 3 --warmup 1 --no-cpu-baseline
step rocprof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --scene scenes/CBlucy_standin.dae --width 1920 --height 1080 --spp 128 --max-depth 8 --envmap synth:1024x512 --rr --steps 2 --warmup 1 --no-cpu-baseline --no-parity
echo "== done"
