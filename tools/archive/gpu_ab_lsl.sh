#!/bin/bash
# A/B of the slot-direct lane-channel splat atomics (BDPT_LANE_SPLAT) against the product source.
cd "$(dirname "$0")/.." || exit 1
LIBS="build_var_base.so build_var_lsl.so" ROUNDS=3 CFGS="scenes/CBlucy_standin.dae 1920 1080 8 5 2;c5:scenes/CBlucy_standin.dae 1920 1080 8 8 2;CBgems 960 540 32 7 2" timeout -k 10 800 bash tools/gpu_ab_r04.sh > gpurun_out/ab_lsl.log 2>&1
grep -E "FAIL|STOP|^== r|Msamples" gpurun_out/ab_lsl.log | paste - - | sed "s/ | spl 0//" | cut -c1-170
