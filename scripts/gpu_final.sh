#!/bin/bash
# end-of-round evidence: the full bench.py (driver config), then the GPU suite
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_bench.log 2> gpurun_out/final_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; exit $rc
