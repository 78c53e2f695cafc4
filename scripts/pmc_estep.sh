#!/bin/bash
# PMC counters of the fused E-step kernels (one counter pass per rocprofv3
# run; kernel-trace only).  usage: scripts/pmc_estep.sh PREC [N]
set -e
PREC=${1:-fp32}
N=${2:-2000000}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$PREC
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d $OUT/a -o a -- python3 benchmarks/estep_micro.py --prec $PREC --iters 2 --n $N
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE \
  -d $OUT/b -o b -- python3 benchmarks/estep_micro.py --prec $PREC --iters 2 --n $N
