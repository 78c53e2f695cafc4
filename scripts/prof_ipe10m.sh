#!/bin/bash
# IPE at the headline shape (10M x 256, k = 1024): bench.py's IPE extra under
# a kernel trace; per-kernel table and the last step's kernel sequence
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d /tmp/p_ipe10 -o r -- \
  python3 bench.py --steps 3 --warmup 1 --no-qpca --no-fit --no-hard --no-mnist --no-pipeline \
  --no-share8 --ipe-steps 3 > gpurun_out/prof_ipe10m.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $(find /tmp/p_ipe10 -name '*.db') --top 25 > gpurun_out/prof_ipe10m.md
python3 scripts/prof_timeline.py /tmp/p_ipe10 --marker ipe16_prep --last 2 --seq-all > gpurun_out/prof_ipe10m_timeline.md
rm -rf /tmp/p_ipe10
echo done
