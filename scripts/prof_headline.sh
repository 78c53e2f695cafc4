#!/bin/bash
# headline q-means step: kernel trace of bench.py with the extras off
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=scripts/pmc_summary.py
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_head -o r -- \
  python3 bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline \
  --steps 20 --warmup 5 > gpurun_out/prof_head.log 2>&1 || exit 1
python3 $S $(find /tmp/p_head -name '*.db') --top 30 > gpurun_out/prof_head.md
python3 scripts/prof_timeline.py /tmp/p_head --marker bounds_filter --first 0 --last 40 > gpurun_out/prof_head_timeline.md
for i in 20 21; do python3 scripts/prof_timeline.py /tmp/p_head --marker bounds_filter --first $i --last 1 > gpurun_out/prof_head_iv$i.md; done
rm -rf /tmp/p_head
echo done
