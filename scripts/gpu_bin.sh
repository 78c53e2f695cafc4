#!/bin/bash
# ipe16 binomial fire draw: law / skip tests, 10M bench, hazard-target sweep
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ipe16_gpu.py tests/test_ipe16_skip_gpu.py tests/test_dmeans_pinned_gpu.py > gpurun_out/b_tests.log 2>&1
rc=$?; echo "ipe tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for ht in 9e-4 4e-4 2e-4; do
  SQ_IPE16_HT=$ht timeout -k 10 240 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 6 > gpurun_out/b_ht_$ht.log 2>&1
  rc=$?; echo "ht $ht rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
