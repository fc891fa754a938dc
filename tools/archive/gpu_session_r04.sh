#!/bin/bash
# Round-4 GPU session. PART=check: host probe, the round-4 GPU tests, the binding's tile loop and
# the reference's render loop through the binding at the north-star frame, a C2 bench line with the
# new parity leg. PART=tests: the whole `pytest -m gpu` suite. PART=bench: bench.py on the
# BASELINE workloads (+ rocprofv3 kernel stats of the default one with ROCPROF=1).
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r04}
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
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [ "${PART:-check}" = check ]; then
  step host 30 bash -c 'nproc; python3 -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; cat /proc/cpuinfo | grep "model name" | head -1'
  step t_fp64 600 $PYT tests/test_fp64_agreement.py -m gpu
  step t_multirank 900 $PYT tests/test_gpu_multirank.py
  step t_integration 600 $PYT tests/test_integration.py -m gpu
  step t_knobs 600 $PYT tests/test_gpu_parity.py -k knobs
  step loop_B_ns 600 oracle/_ref/ref_driver_amd -B -t 16 -s 16 -m 5 -r 1920 1080 scenes/CBlucy_standin.dae
  step loop_B_ns128 600 oracle/_ref/ref_driver_amd -B -t 16 -s 128 -m 5 -r 1920 1080 scenes/CBlucy_standin.dae
  step bench_ns16 600 python bench.py --spp 16 --steps 3 --no-cpu-baseline --no-parity
  step loop_A_ns 900 oracle/_ref/ref_driver_amd -A -t 16 -s 16 -m 5 -r 1920 1080 -f $OUT/loop_a.png scenes/CBlucy_standin.dae
  step bench_c2 900 python bench.py --workload c2
fi
if [ "${PART}" = tests ]; then
  step pytest_gpu 1100 $PYT tests -m gpu
fi
if [ "${PART}" = full ]; then   # the round's record: GPU tests, then every BASELINE workload's bench line
  step pytest_gpu 600 $PYT tests -m gpu
  PART=bench
fi
if [ "${PART}" = bench ]; then
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
