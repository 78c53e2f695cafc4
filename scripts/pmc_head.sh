#!/bin/bash
# PMC of the headline's steady-state kernels (bounds filter, gap screen,
# delta walk): two passes over a short headline-only bench.py run
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
B="bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --no-share8 --steps 5 --warmup 20"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES \
  GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY \
  -d /tmp/p_hp -o r -- python3 $B > gpurun_out/pmc_head.log 2>&1 || exit 1
python3 $S $(find /tmp/p_hp -name '*.db') --match 'bounds_filter|gap_screen|delta_|recheck_fast' --top 8 > gpurun_out/pmc_head.md
rm -rf /tmp/p_hp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
  GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS \
  -d /tmp/p_hp2 -o r -- python3 $B > gpurun_out/pmc_head2.log 2>&1 || exit 1
python3 $S $(find /tmp/p_hp2 -name '*.db') --match 'bounds_filter|gap_screen|delta_|recheck_fast' --top 8 > gpurun_out/pmc_head2.md
rm -rf /tmp/p_hp2
echo done
