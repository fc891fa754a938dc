#!/bin/bash
# Round-3 GPU session. PART=bench: bench.py on every BASELINE workload + the rocprofv3 kernel stats
# of the default one. PART=pmc: per workload, FETCH_SIZE and WRITE_SIZE passes (each with its
# kernel trace, so the bytes carry a duration) -> traffic_<key>.json; SQ and TCC passes for
# WORKLOADS_SQ. One rocprofv3 run per counter group, each under its own time limit.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r03}
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
declare -A ARGS=(
  [ns]="scenes/CBlucy_standin.dae 1920 1080 128 5 1"
  [c2]="scenes/CBspheres.dae 480 360 128 5 1"
  [c3]="scenes/CBlucy_standin.dae 800 600 128 5 1"
  [c4]="scenes/CBgems.dae 1920 1080 256 7 1"
  [c5]="scenes/CBlucy_standin.dae 1920 1080 1024 8 1"
)
declare -A DESC=(
  [ns]="CBlucy stand-in 1920x1080 s128 m5, one launch (tools/prof_render.py)"
  [c2]="CBspheres 480x360 s128 m5, one launch (tools/prof_render.py)"
  [c3]="CBlucy stand-in 800x600 s128 m5, one launch (tools/prof_render.py)"
  [c4]="CBgems 1920x1080 s256 m7, one launch (tools/prof_render.py)"
  [c5]="CBlucy stand-in + synthetic 1024x512 sky 1920x1080 s1024 m8 RR, one launch (tools/prof_render.py)"
)
envs() {  # the C5 stand-in's environment light and roulette for tools/prof_render.py
  if [ "$1" = c5 ]; then export BDPT_ENV=synth:1024x512 BDPT_RR=1; else unset BDPT_ENV BDPT_RR; fi
}
if [ "${PART:-bench}" = bench ]; then
  for w in ${WORKLOADS:-ns c2 c3 c4 c5}; do
    extra=""; [ "$w" != ns ] && extra="--no-cpu-baseline"
    [ "$w" = c4 ] || [ "$w" = c5 ] && extra="$extra --steps 2"
    step bench_$w 900 python bench.py --workload $w $extra
  done
  if [ -n "$ROCPROF" ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity
  fi
fi
if [ "${PART:-bench}" = pmc ]; then
  for w in ${WORKLOADS:-ns c2 c3 c4 c5}; do
    mkdir -p $OUT/$w
    envs $w
    step pmc_fetch_$w 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/$w/pmc_fetch -o run -- python3 tools/prof_render.py ${ARGS[$w]}
    step pmc_write_$w 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/$w/pmc_write -o run -- python3 tools/prof_render.py ${ARGS[$w]}
    step traffic_$w 60 python3 tools/pmc_traffic.py $OUT/$w $w "${DESC[$w]}"
  done
  for w in ${WORKLOADS_SQ:-c3 c5}; do
    envs $w
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
               "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU" \
               "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
      i=$((i+1))
      step sq${i}_$w 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/$w/sq$i -o run -- python3 tools/prof_render.py ${ARGS[$w]}
    done
    python3 tools/pmc_summary.py $OUT/$w/sq1 $OUT/$w/sq2 $OUT/$w/sq3 $OUT/$w/sq4 > $OUT/pmc_$w.txt
    cat $OUT/pmc_$w.txt
  done
fi
echo "== done"
