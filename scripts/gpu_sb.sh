#!/bin/bash
# native skip bounds (ipe16 op 5): tests, then the 10M IPE bench with the
# native and the torch bounds, then the first-step host profile
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ipe16_skip_gpu.py tests/test_ipe16_gpu.py tests/test_ipe16_law_10m_gpu.py > gpurun_out/sb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for nb in 1 0; do
  SQ_IPE16_NATIVE_BOUNDS=$nb timeout -k 10 240 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/sb_bench_$nb.log 2>&1
  rc=$?; echo "bench native=$nb rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 python -u benchmarks/ipe_first_step_profile.py > gpurun_out/sb_first.log 2>&1
rc=$?; echo "first rc=$rc"; exit $rc
