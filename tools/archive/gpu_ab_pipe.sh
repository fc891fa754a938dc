#!/bin/bash
# Parity tests on both pipelines, then megakernel vs wavefront timing.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for pipe in 1 2; do
  BDPT_PIPELINE=$pipe timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_pytest.log; if [ $rc -gt 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
done
for sc in "CBspheres 480 360 128 5 2" "CBgems 480 360 64 5 2" "CBempty 480 360 128 5 2"; do
  for pipe in 1 2; do
    echo "== $sc pipeline=$pipe"
    BDPT_PIPELINE=$pipe timeout -k 10 300 python3 tools/prof_render.py $sc || { echo "STOP rc=$?"; exit 1; }
  done
done
