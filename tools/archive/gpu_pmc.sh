#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; no tracing domains combined with --pmc).
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${PMC_TAG:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
ARGS=${ARGS:-"CBspheres 480 360 32 5 1"}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/prof_render.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 3 $OUT/p$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then grep -qi "counter" $OUT/p$i.log || { echo STOP; exit $rc; }; fi
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_INSTS_VALU_TRANS_F SQ_INSTS_VALU_FMA_F SQ_INSTS_VALU_MUL_F SQ_INSTS_VALU_ADD_F SQ_INSTS_VALU_INT SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VALU_CVT
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GRBM_GUI_ACTIVE SQ_INSTS_FLAT SQ_INSTS_SCRATCH
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS
GROUPS
echo "== done"
