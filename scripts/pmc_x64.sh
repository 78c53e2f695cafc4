#!/bin/bash
# PMC of the certified full-sweep E-step (estep_x64_kernel, 2M x 256, k = 1024):
# MFMA busy, VALU / MFMA, wait shares (two counter passes)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
A="benchmarks/estep_micro.py --prec x64 --iters 3 --n 2000000"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d /tmp/p_x64a -o r -- python3 $A > gpurun_out/pmc_x64a.log 2>&1 || exit 1
python3 $S $(find /tmp/p_x64a -name '*.db') --match estep_x64 --top 4 > gpurun_out/pmc_x64a.md
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
  -d /tmp/p_x64b -o r -- python3 $A > gpurun_out/pmc_x64b.log 2>&1 || exit 1
python3 $S $(find /tmp/p_x64b -name '*.db') --match estep_x64 --top 4 > gpurun_out/pmc_x64b.md
rm -rf /tmp/p_x64a /tmp/p_x64b
echo done
