#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ipe16_skip_gpu.py tests/test_ipe16_gpu.py > gpurun_out/w_tests.log 2>&1
rc=$?; echo "ipe tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 8 > gpurun_out/w_ipe_bench.log 2>&1
rc=$?; echo "ipe bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/c1_touched.py > gpurun_out/w_c1.log 2>&1
rc=$?; echo "c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo done
