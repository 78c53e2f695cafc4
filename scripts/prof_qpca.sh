#!/bin/bash
# qPCA 10M x 256 fits: host phase timings (synchronised) + kernel trace
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
SQ_QPCA_PHASES=1 timeout -k 10 200 python3 benchmarks/qpca_bench.py --solver full > gpurun_out/qpca_full_phases.log 2>&1 || exit 1
SQ_QPCA_PHASES=1 timeout -k 10 200 python3 benchmarks/qpca_bench.py --solver randomized > gpurun_out/qpca_rand_phases.log 2>&1 || exit 1
SQ_QPCA_PHASES=1 timeout -k 10 200 python3 benchmarks/qpca_bench.py --solver full --true-tomography > gpurun_out/qpca_full_tt_phases.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d /tmp/p_qpca -o r -- \
  python3 benchmarks/qpca_bench.py --solver full > gpurun_out/prof_qpca.log 2>&1 || exit 1
python3 $S $(find /tmp/p_qpca -name '*.db') --top 25 > gpurun_out/prof_qpca.md
rm -rf /tmp/p_qpca
echo done
