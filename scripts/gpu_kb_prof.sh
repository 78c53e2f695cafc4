#!/bin/bash
# kernel table of the batched k-means++ restarts (10 restarts, 10M x 256, k = 1024)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p_kb -o r -- python3 benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/kbp_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $(find /tmp/p_kb -name '*.db') --top 25 > gpurun_out/kbp_prof.md
rm -rf /tmp/p_kb
echo done
