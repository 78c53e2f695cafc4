#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_kmpp_batch_gpu.py > gpurun_out/kb2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 400 python -u benchmarks/kmpp_batch_bench.py > gpurun_out/kb2_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
