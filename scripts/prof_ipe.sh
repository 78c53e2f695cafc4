#!/bin/bash
# IPE E-step profile: kernel trace + 2 PMC passes (2M rows)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
A="benchmarks/ipe_bench.py --rows 2000000 --steps 1"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d /tmp/p_ipe_pmc -o r -- python3 $A > gpurun_out/prof_ipe_pmc.log 2>&1 || exit 1
python3 $S $(find /tmp/p_ipe_pmc -name '*.db') --match ipe_fused --top 6 > gpurun_out/prof_ipe_pmc.md
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAIT_ANY \
  -d /tmp/p_ipe_pmc2 -o r -- python3 $A > gpurun_out/prof_ipe_pmc2.log 2>&1 || exit 1
python3 $S $(find /tmp/p_ipe_pmc2 -name '*.db') --match ipe_fused --top 6 > gpurun_out/prof_ipe_pmc2.md
rm -rf /tmp/p_ipe_pmc /tmp/p_ipe_pmc2
echo done
