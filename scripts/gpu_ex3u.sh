#!/bin/bash
# batched k-means++ vs the exact pass's row loads in flight (SQ_KMPP_EX3_U)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for u in 8 16 4; do
  SQ_KMPP_EX3_U=$u timeout -k 10 200 python -u benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/ex3u_$u.log 2>&1
  rc=$?; echo "u=$u rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/ex3u_$u.log
done
