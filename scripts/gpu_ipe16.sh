#!/bin/bash
# ipe16 bring-up: its GPU tests, then the IPE bench at 2M rows
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ipe16_gpu.py > gpurun_out/ipe16_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u benchmarks/ipe_bench.py --rows 2000000 --steps 3 > gpurun_out/ipe16_bench.log 2>&1
echo "bench rc=$?"
