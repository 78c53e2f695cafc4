#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmpp_batch_gpu.py > gpurun_out/sd_kmpp_tests.log 2>&1
rc=$?; echo "kmpp tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ipe16_gpu.py tests/test_ipe16_skip_gpu.py tests/test_ipe_fused_gpu.py tests/test_dmeans_pinned_gpu.py > gpurun_out/sd_ipe_tests.log 2>&1
rc=$?; echo "ipe tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u benchmarks/ipe16_skip_diag.py 10000000 256 1024 9 > gpurun_out/sd_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 8 > gpurun_out/sd_ipe_bench.log 2>&1
rc=$?; echo "ipe bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p_kb -o r -- python3 benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/sd_kbp_run.log 2>&1
rc=$?; echo "kmpp prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $(find /tmp/p_kb -name '*.db') --top 12 > gpurun_out/sd_kbp_prof.md
rm -rf /tmp/p_kb
echo done
