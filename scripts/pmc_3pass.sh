#!/bin/bash
# PMC of the dense-row 3-pass kernels (estep_f32_kernel<16, 2 / 3>) on the
# hard regime (2M x 256, k = 1024, 1024 overlapping blobs): MFMA busy, VALU
# per MFMA, wait shares, scratch (spill) traffic
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
timeout -s KILL 200 rocprofv3 --kernel-trace --kernel-include-regex estep_f32 --pmc SQ_INSTS_MFMA \
  SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY \
  SQ_INSTS_LDS -d /tmp/p_3p -o r -- python3 benchmarks/hard_bench.py > gpurun_out/pmc_3p.log 2>&1 || exit 1
python3 $S $(find /tmp/p_3p -name '*.db') --match estep_f32 --top 4 > gpurun_out/pmc_3p.md
rm -rf /tmp/p_3p
echo done
