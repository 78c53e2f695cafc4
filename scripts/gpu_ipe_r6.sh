#!/bin/bash
# ipe16 at 10M x 256, k = 1024 (bench shape): IPE bench, kernel trace of the
# steady state, and two PMC passes over the final ipe16 kernels
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
A="benchmarks/ipe_bench.py --rows 10000000 --steps 8"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_ipe6 -o r -- python3 $A > gpurun_out/ipe6_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_timeline.py /tmp/p_ipe6 --marker ipe16_prep --last 6 --seq-all > gpurun_out/ipe6_timeline.md
python3 scripts/pmc_summary.py $(find /tmp/p_ipe6 -name '*.db') --top 25 > gpurun_out/ipe6_prof.md
rm -rf /tmp/p_ipe6
S=scripts/pmc_summary.py
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d /tmp/p_i6a -o r -- python3 $A > gpurun_out/ipe6_pmca.log 2>&1 || exit 1
python3 $S $(find /tmp/p_i6a -name '*.db') --match ipe16 --top 6 > gpurun_out/ipe6_pmca.md
rm -rf /tmp/p_i6a
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD \
  -d /tmp/p_i6b -o r -- python3 $A > gpurun_out/ipe6_pmcb.log 2>&1 || exit 1
python3 $S $(find /tmp/p_i6b -name '*.db') --match ipe16 --top 6 > gpurun_out/ipe6_pmcb.md
rm -rf /tmp/p_i6b
echo done
