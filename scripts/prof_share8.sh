#!/bin/bash
# N = 8 per-GPU share (1.25M rows) of the headline step: kernel trace + timeline
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_s8 -o r -- \
  python3 bench.py --rows 1250000 --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline \
  --steps 20 --warmup 5 > gpurun_out/prof_s8.log 2>&1 || exit 1
python3 scripts/prof_timeline.py /tmp/p_s8 --marker bounds_filter --first 0 --last 40 > gpurun_out/prof_s8_timeline.md
for i in 15 16; do python3 scripts/prof_timeline.py /tmp/p_s8 --marker bounds_filter --first $i --last 1 > gpurun_out/prof_s8_iv$i.md; done
rm -rf /tmp/p_s8
echo done
