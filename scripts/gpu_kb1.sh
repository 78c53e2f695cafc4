#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kmpp_batch_gpu.py tests/test_kmpp_gpu.py tests/test_dmeans_pinned_gpu.py tests/test_pipeline_gpu.py tests/test_device_estimators_gpu.py > gpurun_out/kb1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/kb1_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
