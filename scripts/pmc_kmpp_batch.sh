#!/bin/bash
# PMC of the batched k-means++ kernels (10 restarts, 10M x 256, k = 256 to keep the run short)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES \
  GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY \
  -d /tmp/p_kbp -o r -- python3 benchmarks/kmpp_batch_bench.py 10000000 256 10 \
  > gpurun_out/pmc_kb.log 2>&1 || exit 1
python3 $S $(find /tmp/p_kbp -name '*.db') --match kmpp_ --top 8 > gpurun_out/pmc_kb.md
rm -rf /tmp/p_kbp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
  SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY \
  -d /tmp/p_kbp2 -o r -- python3 benchmarks/kmpp_batch_bench.py 10000000 256 10 \
  > gpurun_out/pmc_kb2.log 2>&1 || exit 1
python3 $S $(find /tmp/p_kbp2 -name '*.db') --match kmpp_ --top 8 > gpurun_out/pmc_kb2.md
rm -rf /tmp/p_kbp2
echo done
