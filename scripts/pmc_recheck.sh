#!/bin/bash
# PMC counters of the fp64 re-check (multi-candidate rows) on the bench
# data: scripts/churn.py drives 15 Lloyd iterations; one counter pass per
# rocprofv3 run, kernel-trace only, limited to the re-check kernel.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_recheck
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex recheck \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM \
  SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE \
  -d $OUT/a -o a -- python3 scripts/churn.py > $OUT/a.log 2>&1
timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex recheck \
  --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
  -d $OUT/b -o b -- python3 scripts/churn.py > $OUT/b.log 2>&1
python3 scripts/pmc_summary.py $OUT/a/a_results.db $OUT/b/b_results.db --match recheck > $OUT/summary.md
rm -rf $OUT/a $OUT/b
