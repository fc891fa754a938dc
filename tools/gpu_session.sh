#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace of the bench command,
# then FETCH_SIZE / WRITE_SIZE passes (separate runs, no tracing domains) on one bench-sized launch.
# Stops at the first crash/timeout (exit codes other than 0/1 from a step).
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
  tail -n 30 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > $OUT/smi.log 2>&1 || true
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 1200 python -m pytest tests -m gpu -x -q -s
  step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 900 python bench.py --steps 5 --warmup 1
step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity
# one C2 launch (128 spp) per run; the warm-up launch (1 spp) is a separate dispatch
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 tools/prof_render.py CBspheres 480 360 128 5 1
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 tools/prof_render.py CBspheres 480 360 128 5 1
step pmc_l2 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_l2 -o run -- python3 tools/prof_render.py CBspheres 480 360 128 5 1
echo "== done"
