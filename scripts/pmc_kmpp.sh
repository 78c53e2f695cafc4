#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES \
  GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY \
  -d /tmp/p_kp -o r -- python3 benchmarks/kmpp_bench.py --k 256 --center --no-unpruned \
  > gpurun_out/pmc_kmpp.log 2>&1 || exit 1
python3 $S $(find /tmp/p_kp -name '*.db') --match kmpp_ --top 8 > gpurun_out/pmc_kmpp.md
rm -rf /tmp/p_kp
echo done
