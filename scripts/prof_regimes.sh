#!/bin/bash
# headline bench's unpruned / first-iteration regimes: kernel sequences of the
# last E-step-to-E-step intervals (unpruned steps, then the first iteration)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_reg -o r -- \
  python3 bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline \
  --steps 5 --warmup 2 > gpurun_out/prof_reg.log 2>&1 || exit 1
python3 scripts/prof_timeline.py /tmp/p_reg --marker estep_x64 --last 14 --seq-all > gpurun_out/prof_reg_timeline.md
rm -rf /tmp/p_reg
echo done
