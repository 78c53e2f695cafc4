#!/bin/bash
# ipe16 tests + 10M IPE bench
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ipe16_gpu.py tests/test_ipe16_skip_gpu.py tests/test_ipe16_wide_gpu.py tests/test_ipe16_law_10m_gpu.py tests/test_ipe_fused_gpu.py tests/test_dmeans_pinned_gpu.py > gpurun_out/i16t_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/i16t_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
