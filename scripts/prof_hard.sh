#!/bin/bash
# hard regime (overlapping blobs, 2M rows): kernel table + the kernel sequence
# of the last steady-state steps
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_hard -o r -- \
  python3 benchmarks/hard_bench.py > gpurun_out/prof_hard.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $(find /tmp/p_hard -name '*.db') --top 30 > gpurun_out/prof_hard.md
python3 scripts/prof_timeline.py /tmp/p_hard --marker estep_x64 --last 3 --seq-all > gpurun_out/prof_hard_timeline.md
rm -rf /tmp/p_hard
echo done
