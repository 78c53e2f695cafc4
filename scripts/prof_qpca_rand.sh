#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d /tmp/p_qr -o r -- \
  python3 benchmarks/qpca_bench.py --solver randomized > gpurun_out/prof_qpca_rand.log 2>&1 || exit 1
python3 $S $(find /tmp/p_qr -name '*.db') --top 16 > gpurun_out/prof_qpca_rand.md
rm -rf /tmp/p_qr
echo done
