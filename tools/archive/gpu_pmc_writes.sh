#!/bin/bash
# Where the north star's HBM-side writes come from: EA write requests split into atomics and
# 32 / 64-B writes, L2 write-backs, and the store / atomic instruction counts (one pass each).
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${PMC_TAG:-pmcw}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:-"scenes/CBlucy_standin.dae 1920 1080 8 5 1"}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/prof_render.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 $OUT/p$i.log
  if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi
done <<GROUPS
TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
TCC_ATOMIC_sum TCC_WRITEBACK_sum
SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_WAVES
WRITE_SIZE
GROUPS
echo "== done"
