#!/bin/bash
# ipe16 law tests + skip tests, then bench.py's IPE extra alone
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ipe16_gpu.py tests/test_ipe16_skip_gpu.py > gpurun_out/ipeb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-qpca --no-fit --no-hard --no-mnist --no-pipeline --no-share8 > gpurun_out/ipeb_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
