#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_ipe16_skip_gpu.py tests/test_ipe16_law_10m_gpu.py tests/test_ipe16_gpu.py > gpurun_out/fs2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_first_step_profile.py > gpurun_out/fs2.log 2>&1
rc=$?; echo "fsp rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 8 > gpurun_out/fs2_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
