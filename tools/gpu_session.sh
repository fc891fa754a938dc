#!/bin/bash
# The GPU session script (round 5 onward; the earlier per-round scripts were removed in round 6, git history has them).
#   PART=tests    the whole `pytest -m gpu` suite
#   PART=phases   phase split + lane use per phase (BDPT_PHASE_PROF variants build_var_ph.so (m <= 5)
#                 and build_var_ph8.so (m <= 8), tools/build_variants.sh) on the north star and C5
#   PART=bench    bench.py on WORKLOADS (default: ns c2 c3 c4 c5); ROCPROF=1 adds the rocprofv3
#                 kernel stats of the default line
#   PART=pmc      FETCH_SIZE / WRITE_SIZE passes per workload -> traffic_<w>.json, SQ / TCC groups
#                 for WORKLOADS_SQ (default ns c5)
#   PART=ab       A/B of variant libraries: LIBS="build_var_a.so build_var_b.so ..." on CFGS
#                 (prof_render.py argument strings separated by ';'), ROUNDS interleaved rounds
#   PART=pt       bench.py --integrator pt (the PathTracer) on ns, c2, a microfacet scene, bunny.dae
#   PART=full     tests, then bench
# Every GPU step runs under its own timeout; the script stops at the first abort / fault / timeout.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r06}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n ${TAIL:-3} "$OUT/$name.log" | cut -c1-3000
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
PART=${PART:-tests}
if [ "$PART" = tests ] || [ "$PART" = full ]; then
  step pytest_gpu 1000 $PYT tests -m gpu
fi
if [ "$PART" = phases ]; then
  TAIL=30
  step ph_ns 300 env BDPT_LIB=$PWD/build_var_ph.so BDPT_PHASES=1 python3 tools/prof_render.py scenes/CBlucy_standin.dae 1920 1080 8 5 1
  step ph_c5 300 env BDPT_LIB=$PWD/build_var_ph8.so BDPT_PHASES=1 BDPT_ENV=synth:1024x512 BDPT_RR=1 python3 tools/prof_render.py scenes/CBlucy_standin.dae 1920 1080 8 8 1
  step ph_c2 300 env BDPT_LIB=$PWD/build_var_ph.so BDPT_PHASES=1 python3 tools/prof_render.py CBspheres 480 360 32 5 1
  step ph_c4 300 env BDPT_LIB=$PWD/build_var_ph8.so BDPT_PHASES=1 python3 tools/prof_render.py scenes/CBgems.dae 1920 1080 8 7 1
fi
if [ "$PART" = ab ]; then
  IFS=';' read -ra cfgs <<< "${CFGS:-scenes/CBlucy_standin.dae 1920 1080 32 5 2}"
  for r in $(seq 1 ${ROUNDS:-2}); do
    for c in "${cfgs[@]}"; do
      for lib in $LIBS; do
        # leading KEY=VAL words are environment (e.g. BDPT_LDS_MODE=0); "c5" = the C5 shape
        # (synthetic sky + roulette)
        envx=""; a=""
        for wd in $c; do
          if [ -z "$a" ] && [[ "$wd" == *=* ]]; then envx="$envx $wd"
          elif [ -z "$a" ] && [ "$wd" = c5 ]; then envx="$envx BDPT_ENV=synth:1024x512 BDPT_RR=1"
          else a="$a $wd"; fi
        done
        step ab_r${r}_$(basename $lib .so)_$(echo $c | tr ' /.' '___') 300 env BDPT_LIB=$PWD/$lib $envx python3 tools/prof_render.py $a
      done
    done
  done
fi
if [ "$PART" = pmc ]; then
  # per workload: FETCH_SIZE and WRITE_SIZE passes (each with its kernel trace, so the bytes carry a
  # duration) -> $OUT/<w>/traffic_<w>.json; then the SQ / TCC groups for WORKLOADS_SQ. One rocprofv3
  # run per counter group (never combined with tracing domains), each under its own time limit.
  declare -A ARGS=([ns]="scenes/CBlucy_standin.dae 1920 1080 128 5 1" [c2]="scenes/CBspheres.dae 480 360 128 5 1"
    [c3]="scenes/CBlucy_standin.dae 800 600 128 5 1" [c4]="scenes/CBgems.dae 1920 1080 256 7 1"
    [c5]="scenes/CBlucy_standin.dae 1920 1080 1024 8 1")
  declare -A DESC=([ns]="CBlucy stand-in 1920x1080 s128 m5" [c2]="CBspheres 480x360 s128 m5"
    [c3]="CBlucy stand-in 800x600 s128 m5" [c4]="CBgems 1920x1080 s256 m7"
    [c5]="CBlucy stand-in + synthetic 1024x512 sky 1920x1080 s1024 m8 RR")
  envs() { if [ "$1" = c5 ]; then export BDPT_ENV=synth:1024x512 BDPT_RR=1; else unset BDPT_ENV BDPT_RR; fi; }
  for w in ${WORKLOADS:-ns c2 c3 c4 c5}; do
    mkdir -p $OUT/$w
    envs $w
    step pmc_fetch_$w 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/$w/pmc_fetch -o run -- python3 tools/prof_render.py ${ARGS[$w]}
    step pmc_write_$w 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/$w/pmc_write -o run -- python3 tools/prof_render.py ${ARGS[$w]}
    step traffic_$w 60 python3 tools/pmc_traffic.py $OUT/$w $w "${DESC[$w]}, one launch (tools/prof_render.py)"
  done
  for w in ${WORKLOADS_SQ:-ns c5}; do
    envs $w
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
               "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU" \
               "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      step sq${i}_$w 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/$w/sq$i -o run -- python3 tools/prof_render.py ${ARGS[$w]}
    done
    python3 tools/pmc_summary.py $OUT/$w/sq1 $OUT/$w/sq2 $OUT/$w/sq3 > $OUT/pmc_$w.txt
    cat $OUT/pmc_$w.txt
  done
fi
if [ "$PART" = pt ]; then
  # the unidirectional PathTracer on the BDPT workloads' scenes and the ones only it renders
  step bench_pt_ns 600 python bench.py --integrator pt --workload ns --steps 3 --warmup 1 --no-cpu-baseline
  step bench_pt_c2 600 python bench.py --integrator pt --workload c2 --steps 3 --warmup 1 --no-cpu-baseline
  step bench_pt_mf 600 python bench.py --integrator pt --scene scenes/CBspheres_microfacet_al_ag.dae --steps 3 --warmup 1 --no-cpu-baseline
  step bench_pt_bunny 600 python bench.py --integrator pt --scene scenes/bunny.dae --steps 3 --warmup 1 --no-cpu-baseline
  if [ -n "$ROCPROF" ]; then
    step rocprof_pt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pt -o run -- python3 bench.py --integrator pt --steps 3 --warmup 1 --no-cpu-baseline --no-parity
  fi
fi
if [ "$PART" = bench ] || [ "$PART" = full ]; then
  for w in ${WORKLOADS:-ns c2 c3 c4 c5}; do
    extra=""; [ "$w" != ns ] && extra="--no-cpu-baseline"
    [ "$w" = c4 ] || [ "$w" = c5 ] && extra="$extra --steps 2"
    step bench_$w 900 python bench.py --workload $w $extra
  done
  if [ -n "$ROCPROF" ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity
  fi
fi
echo "== done"
