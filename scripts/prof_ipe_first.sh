#!/bin/bash
# IPE first steps (no label hints yet): per-step screen statistics and the kernel table
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1 PYTHONPATH=.
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_if -o r -- \
  python3 benchmarks/ipe_bench.py --steps 2 > gpurun_out/prof_ipe_first.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $(find /tmp/p_if -name '*.db') --top 12 > gpurun_out/prof_ipe_first.md
rm -rf /tmp/p_if
echo done
