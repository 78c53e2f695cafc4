#!/bin/bash
# ipe16 kernel table over Lloyd steps (1M rows by default)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
ROWS=${1:-1000000}
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p_i16 -o r -- \
  python3 benchmarks/ipe16_steps.py $ROWS 8 > gpurun_out/prof_ipe16.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $(find /tmp/p_i16 -name '*.db') --top 25 > gpurun_out/prof_ipe16.md
python3 scripts/prof_timeline.py /tmp/p_i16 --marker ipe16_prep --last 2 --seq-all > gpurun_out/prof_ipe16_timeline.md
rm -rf /tmp/p_i16
echo done
