#!/bin/bash
# kernel timeline of the final IPE step (10M x 256, k = 1024, one launch group)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_if -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/if_prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_timeline.py /tmp/p_if --marker ipe16_prep --last 3 --seq-all > gpurun_out/if_timeline.md
rm -rf /tmp/p_if
echo done
