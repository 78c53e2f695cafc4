#!/bin/bash
# ipe16 with every row's fires finished in prep: law / skip tests, 10M bench
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ipe16_gpu.py tests/test_ipe16_skip_gpu.py > gpurun_out/pf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 8 > gpurun_out/pf_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_pf -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 4 > gpurun_out/pf_prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_timeline.py /tmp/p_pf --marker ipe16_prep --last 6 --seq-all > gpurun_out/pf_timeline.md
rm -rf /tmp/p_pf
echo done
