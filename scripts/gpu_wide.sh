#!/bin/bash
# ipe16 for wide rows: values-pass bit identity, law at d = 784 / 1000, MNIST shape
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ipe16_wide_gpu.py > gpurun_out/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ipe16_gpu.py tests/test_ipe16_skip_gpu.py > gpurun_out/wide_ipe16_tests.log 2>&1
rc=$?; echo "ipe16 tests rc=$rc"; exit $rc
