#!/bin/bash
# kernel timeline of the first two IPE steps (10M x 256, k = 1024, random-row centres)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_sp -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 1 > gpurun_out/sp_prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_timeline.py /tmp/p_sp --marker ipe16_prep --last 2 --seq-all > gpurun_out/sp_timeline.md
rm -rf /tmp/p_sp
echo done
