#!/bin/bash
# PMC of the ipe16 kernels (sweep / prep / near) over Lloyd steps at 1M rows
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
A="benchmarks/ipe16_steps.py ${1:-1000000} 5"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d /tmp/p_i16a -o r -- python3 $A > gpurun_out/pmc_i16a.log 2>&1 || exit 1
python3 $S $(find /tmp/p_i16a -name '*.db') --match ipe16 --top 6 > gpurun_out/pmc_i16a.md
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD \
  -d /tmp/p_i16b -o r -- python3 $A > gpurun_out/pmc_i16b.log 2>&1 || exit 1
python3 $S $(find /tmp/p_i16b -name '*.db') --match ipe16 --top 6 > gpurun_out/pmc_i16b.md
rm -rf /tmp/p_i16a /tmp/p_i16b
echo done
