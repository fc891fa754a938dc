#!/bin/bash
# PMC A/B of library builds: LIBS="a.so b.so" ARGS="scene W H spp M launches"; three passes per
# library (SQ instruction mix / waits, FETCH_SIZE, WRITE_SIZE), one rocprofv3 run each.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${PMC_TAG:-pmcab}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:-"scenes/CBlucy_standin.dae 1920 1080 8 5 1"}
for lib in $LIBS; do
  tag=$(basename $lib .so)
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SCRATCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1)); mkdir -p $OUT/$tag
    echo "== $tag pass $i: $grp"
    BDPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/$tag/p$i -o run -- python3 tools/prof_render.py $ARGS > $OUT/$tag/p$i.log 2>&1 || { echo STOP; tail -5 $OUT/$tag/p$i.log; exit 1; }
    tail -n 1 $OUT/$tag/p$i.log
  done
  python3 tools/pmc_summary.py $OUT/$tag/p1 $OUT/$tag/p2 $OUT/$tag/p3
done
