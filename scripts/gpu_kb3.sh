#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmpp_batch_gpu.py > gpurun_out/kb3_tests.log 2>&1
rc=$?; echo "kmpp tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p_kb -o r -- python3 benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/kb3_run.log 2>&1
rc=$?; echo "kmpp prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $(find /tmp/p_kb -name '*.db') --top 12 > gpurun_out/kb3_prof.md
rm -rf /tmp/p_kb
echo done
