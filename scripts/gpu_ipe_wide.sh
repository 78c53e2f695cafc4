#!/bin/bash
# IPE for every shape: Q <= 31, d_pad 2048 (fused kernels), the IPE GPU suites
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_ipe_fused_gpu.py tests/test_ipe16_gpu.py > gpurun_out/ipe_wide.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/ipe_wide.log | tail -40
exit $rc
