#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ipe16_skip_gpu.py > gpurun_out/skip3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python -u benchmarks/ipe16_skip_diag.py 2000000 256 1024 8 > gpurun_out/skip3_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 3 > gpurun_out/skip3_bench_on.log 2>&1
rc=$?; echo "bench on rc=$rc"; exit $rc
