#!/bin/bash
# k-means++ kernel profile (10M x 256, k = 1024, pruned)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d /tmp/p_kmpp -o r -- \
  python3 benchmarks/kmpp_bench.py --k 1024 --center --no-unpruned > gpurun_out/prof_kmpp.log 2>&1 || exit 1
python3 $S $(find /tmp/p_kmpp -name '*.db') --top 20 > gpurun_out/prof_kmpp.md
rm -rf /tmp/p_kmpp
echo done
