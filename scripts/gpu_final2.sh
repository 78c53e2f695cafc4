#!/bin/bash
# the newest kernels' own tests first, then the full bench.py and the GPU suite
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kmpp_batch_gpu.py > gpurun_out/f2_kmpp_tests.log 2>&1
rc=$?; echo "kmpp tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/f2_kmpp_bench.log 2>&1
rc=$?; echo "kmpp bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_final.sh
