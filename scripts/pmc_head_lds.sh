#!/bin/bash
# LDS instructions and bank conflicts of the headline's and the IPE step's kernels
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
B="bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --no-share8 --steps 5 --warmup 20"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  -d /tmp/p_hl -o r -- python3 $B > gpurun_out/pmc_hl.log 2>&1 || exit 1
python3 $S $(find /tmp/p_hl -name '*.db') --top 12 > gpurun_out/pmc_hl.md
rm -rf /tmp/p_hl
echo done
