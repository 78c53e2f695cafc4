#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ipe16_skip_gpu.py > gpurun_out/skip4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
for sk in 1 0; do
SQ_IPE16_SKIP=$sk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_sk$sk -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/skip4_run$sk.log 2>&1
rc=$?; echo "prof $sk rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_timeline.py /tmp/p_sk$sk --marker ipe16_prep --last 3 --seq-all > gpurun_out/skip4_timeline$sk.md
python3 scripts/pmc_summary.py $(find /tmp/p_sk$sk -name '*.db') --top 25 > gpurun_out/skip4_prof$sk.md
rm -rf /tmp/p_sk$sk
done
echo done
