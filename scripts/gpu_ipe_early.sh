#!/bin/bash
# kernel totals of the first two IPE steps (random-row centres) at 10M
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_e -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 1 > gpurun_out/early_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $(find /tmp/p_e -name '*.db') --top 20 > gpurun_out/early_prof.md
python3 scripts/prof_timeline.py /tmp/p_e --marker ipe16_prep --last 8 > gpurun_out/early_timeline.md
rm -rf /tmp/p_e
echo done
