#!/bin/bash
# ipe16 row skip: its GPU tests, the ipe16 law tests, the skip-edge scan, the
# row-skip diagnostic at the bench shape (stops at the first crash / timeout)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ipe16_skip_gpu.py tests/test_ipe16_gpu.py > gpurun_out/skip_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 200 python -u benchmarks/ipe16_skip_edge.py > gpurun_out/skip_edge.log 2>&1
rc=$?; echo "edge rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python -u benchmarks/ipe16_rowskip_diag.py 10000000 6 > gpurun_out/rowskip_diag2.log 2>&1
rc=$?; echo "diag rc=$rc"; exit $rc
