#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kmeans_gpu.py -k "mu" > gpurun_out/mu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 200 python -u benchmarks/mu_bench.py > gpurun_out/mu_bench.log 2>&1
rc=$?; echo "mu rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
rc=$?; echo "hard rc=$rc"; exit $rc
