#!/bin/bash
# N = 8 per-GPU share (bench.py's share8 extra: 1.25M rows, the headline's
# initial centres): kernel trace, last E-step-to-E-step intervals
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_s8 -o r -- \
  python3 bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline \
  --steps 20 --warmup 5 > gpurun_out/prof_s8.log 2>&1 || exit 1
python3 scripts/prof_timeline.py /tmp/p_s8 --marker bounds_filter --last 6 > gpurun_out/prof_s8_timeline.md
rm -rf /tmp/p_s8
echo done
