#!/bin/bash
# Round-2 GPU session. PART=a: GPU tests, smoke, the default bench (north star), its rocprofv3
# kernel stats and FETCH/WRITE PMC passes of one north-star launch. PART=b: the other BASELINE
# configs and the phase split (BDPT_PHASE_PROF variant, prebuilt as build_var_ph.so).
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n ${TAIL:-3} "$OUT/$name.log" | cut -c1-2500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
NS="scenes/CBlucy_standin.dae 1920 1080 128 5 1"
if [ "${PART:-a}" = a ]; then
  if [ -z "$SKIP_TESTS" ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  fi
  step bench 600 python bench.py
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 tools/prof_render.py $NS
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 tools/prof_render.py $NS
  step traffic 60 python3 tools/pmc_traffic.py $OUT ns "CBlucy stand-in 1920x1080 s128 m5, one launch (tools/prof_render.py)"
  # C2 (the verdict's second traffic case): same passes into their own directories
  C2="CBspheres 480 360 128 5 1"
  mkdir -p $OUT/c2
  step pmc_fetch_c2 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2/pmc_fetch -o run -- python3 tools/prof_render.py $C2
  step pmc_write_c2 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2/pmc_write -o run -- python3 tools/prof_render.py $C2
  step traffic_c2 60 python3 tools/pmc_traffic.py $OUT/c2 c2 "CBspheres 480x360 s128 m5, one launch (tools/prof_render.py)"
fi
if [ "${PART:-a}" = b ]; then
  step bench_c2 600 python bench.py --workload c2 --no-cpu-baseline
  step bench_c3 600 python bench.py --workload c3 --no-cpu-baseline
  step bench_c4 600 python bench.py --workload c4 --steps 2 --no-cpu-baseline
  step bench_c5 900 python bench.py --workload c5 --steps 2 --no-cpu-baseline
  if [ -f build_var_ph.so ]; then
    CFGS="CBspheres 480 360 64 5 1;scenes/CBlucy_standin.dae 1920 1080 8 5 1;CBgems 480 360 32 5 1" step phases 600 bash tools/gpu_phases.sh
  fi
fi
echo "== done"
