#!/bin/bash
# PMC counters of the gap screen vs the fp32 screen on the bench data
# (scripts/churn.py: 15 Lloyd iterations); one counter pass per run.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gap
mkdir -p $OUT
R='gap_screen|recheck_fast'
timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex "$R" \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM \
  GRBM_GUI_ACTIVE -d $OUT/a -o a -- python3 scripts/churn.py > $OUT/a.log 2>&1
timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex "$R" \
  --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
  -d $OUT/b -o b -- python3 scripts/churn.py > $OUT/b.log 2>&1
timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex "$R" \
  --pmc TA_BUSY_avr TD_TD_BUSY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum \
  -d $OUT/c -o c -- python3 scripts/churn.py > $OUT/c.log 2>&1
python3 scripts/pmc_summary.py $OUT/a/a_results.db $OUT/b/b_results.db $OUT/c/c_results.db > $OUT/summary.md
rm -rf $OUT/a $OUT/b $OUT/c
