#!/bin/bash
# A/B of the build_var_*.so variants over several workloads (tools/gpu_ab.sh per workload); one
# log under gpurun_out/, summary lines on stdout.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
LOG=gpurun_out/${AB_LOG:-ab_multi}.log
CFGS=${CFGS:-"CBspheres 480 360 128 5 2;scenes/CBlucy_standin.dae 1920 1080 16 5 2;CBgems 480 360 64 5 2"}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
: > "$LOG"
for a in "${CFG_LIST[@]}"; do
  ARGS="$a" timeout -k 10 400 bash tools/gpu_ab.sh >> "$LOG" 2>&1 || { echo "STOP"; break; }
done
grep -E "^== |Msamples|STOP" "$LOG"
