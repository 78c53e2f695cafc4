#!/bin/bash
# k-means++ fused restarts + exact2, ipe16 prep-finished fires: tests,
# benches, kernel tables
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmpp_batch_gpu.py > gpurun_out/c_kmpp_tests.log 2>&1
rc=$?; echo "kmpp tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ipe16_gpu.py tests/test_ipe16_skip_gpu.py > gpurun_out/c_ipe_tests.log 2>&1
rc=$?; echo "ipe tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/c_kmpp_bench.log 2>&1
rc=$?; echo "kmpp bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 8 > gpurun_out/c_ipe_bench.log 2>&1
rc=$?; echo "ipe bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p_kb -o r -- python3 benchmarks/kmpp_batch_bench.py 10000000 1024 10 > gpurun_out/c_kbp_run.log 2>&1
rc=$?; echo "kmpp prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $(find /tmp/p_kb -name '*.db') --top 16 > gpurun_out/c_kbp_prof.md
rm -rf /tmp/p_kb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_pf -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 4 > gpurun_out/c_ipe_prof_run.log 2>&1
rc=$?; echo "ipe prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_timeline.py /tmp/p_pf --marker ipe16_prep --last 6 --seq-all > gpurun_out/c_ipe_timeline.md
rm -rf /tmp/p_pf
echo done
