#!/bin/bash
# IPE first steps on the bench data (10M rows): per-step ms + screen stats,
# then a kernel trace of the first two steps
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python3 benchmarks/ipe16_steps.py 10000000 4 > gpurun_out/ipe_first_steps.log 2>&1 || exit 1
cat gpurun_out/ipe_first_steps.log | head -6
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_if -o r -- \
  python3 benchmarks/ipe16_steps.py 10000000 2 > gpurun_out/prof_ipe_first.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $(find /tmp/p_if -name '*.db') --top 25 > gpurun_out/prof_ipe_first.md
rm -rf /tmp/p_if
echo done
