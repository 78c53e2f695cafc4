#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/ipe16_skip_diag.py 10000000 256 1024 8 > gpurun_out/i7_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_i7 -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/i7_prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_timeline.py /tmp/p_i7 --marker ipe16_prep --last 6 --seq-all > gpurun_out/i7_timeline.md
rm -rf /tmp/p_i7
echo done
