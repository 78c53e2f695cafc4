#!/bin/bash
# ipe16 row skip with wild centroids: tests, 10M bench (skip on / off), diag
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ipe16_skip_gpu.py tests/test_ipe16_gpu.py > gpurun_out/skip2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 3 > gpurun_out/skip2_bench_on.log 2>&1
rc=$?; echo "bench on rc=$rc"; [ $rc -eq 0 ] || exit $rc
SQ_IPE16_SKIP=0 timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 3 > gpurun_out/skip2_bench_off.log 2>&1
rc=$?; echo "bench off rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe16_skip_diag.py 2000000 256 1024 8 > gpurun_out/skip2_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; exit $rc
