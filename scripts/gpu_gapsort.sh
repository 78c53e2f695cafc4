#!/bin/bash
# ordered list B for the gap screen: exactness tests, headline bench (sort on /
# off), one steady-state kernel sequence with the sort on
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_multi_records_gpu.py tests/test_estep_overflow_gpu.py > gpurun_out/gs_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
for gs in 1 0; do
SQ_GAP_SORT=$gs timeout -k 10 300 python -u bench.py --no-qpca --no-fit --ipe-steps 0 --no-hard --no-mnist --no-pipeline --steps 20 --warmup 5 > gpurun_out/gs_bench$gs.log 2>&1
rc=$?; echo "bench $gs rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/prof_headline.sh
