#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "== pytest_gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -n 25 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP; exit $rc; fi
echo "== ab"; bash tools/gpu_ab.sh 2>&1 | tee $OUT/ab.log | grep -v '^$'
