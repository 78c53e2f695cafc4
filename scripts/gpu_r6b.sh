#!/bin/bash
# fused k-means++ restart passes: tests, bench (fused / per-restart), kernel
# table; then the ipe16 10M profile (scripts/gpu_ipe_r6.sh)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kmpp_batch_gpu.py > gpurun_out/kf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/kf_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
SQ_KMPP_FUSED=0 timeout -k 10 300 python -u benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/kf_bench_off.log 2>&1
rc=$?; echo "bench off rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_kb_prof.sh || exit 1
bash scripts/gpu_ipe_r6.sh
