#!/bin/bash
# batched k-means++ restarts: GPU tests, then bench.py's IPE + fit extras
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_kmpp_batch_gpu.py tests/test_kmpp_gpu.py tests/test_ipe16_skip_gpu.py > gpurun_out/kb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-qpca --no-hard --no-mnist --no-pipeline --no-share8 > gpurun_out/kb_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
