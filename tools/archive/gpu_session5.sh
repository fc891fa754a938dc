#!/bin/bash
# Round-1 v14 session: GPU tests, smoke, the default bench under rocprofv3 stats, the north-star and
# C5 stand-ins, the PathTracer benches, then FETCH/WRITE PMC passes of one C2 launch.
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
  tail -n ${TAIL:-3} "$OUT/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py --steps 5 --warmup 1
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity
step bench_ns 600 python bench.py --scene scenes/CBlucy_standin.dae --width 1920 --height 1080 --spp 128 --max-depth 5 --steps 3 --warmup 1 --no-cpu-baseline
step bench_c3 600 python bench.py --scene scenes/CBlucy_standin.dae --width 800 --height 600 --spp 128 --max-depth 5 --steps 3 --warmup 1 --no-cpu-baseline
step bench_c5 600 python bench.py --scene scenes/CBlucy_standin.dae --width 1920 --height 1080 --spp 128 --max-depth 8 --envmap synth:1024x512 --rr --steps 3 --warmup 1 --no-cpu-baseline
step bench_pt 600 python bench.py --integrator pt --steps 3 --warmup 1 --no-cpu-baseline
step bench_pt_mf 600 python bench.py --integrator pt --scene scenes/CBspheres_microfacet_al_ag.dae --steps 3 --warmup 1 --no-cpu-baseline
step bench_pt_bunny 600 python bench.py --integrator pt --scene scenes/bunny.dae --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 tools/prof_render.py CBspheres 480 360 128 5 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 tools/prof_render.py CBspheres 480 360 128 5 1
echo "== done"
