#!/bin/bash
# exact pair pass: one pair per lane vs two interleaved (SQ_KMPP_EX3_PP), ids checked by the tests
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
SQ_KMPP_EX3_PP=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kmpp_batch_gpu.py > gpurun_out/ex3pp_tests.log 2>&1
rc=$?; echo "pp2 tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for pp in 1 2 1 2; do
  SQ_KMPP_EX3_PP=$pp timeout -k 10 200 python -u benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/ex3pp_$pp.log 2>&1
  rc=$?; echo "pp=$pp rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/ex3pp_$pp.log
done
