#!/bin/bash
# ipe16 pair certificate: law tests, the 10M IPE bench, a kernel trace of it
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ipe16_gpu.py > gpurun_out/cert_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python -u benchmarks/ipe_bench.py --rows 10000000 --steps 3 > gpurun_out/cert_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_cert -o r -- python3 benchmarks/ipe_bench.py --rows 10000000 --steps 2 > gpurun_out/cert_prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $(find /tmp/p_cert -name '*.db') --top 20 > gpurun_out/cert_prof.md
python3 scripts/prof_timeline.py /tmp/p_cert --marker ipe16_prep --last 2 --seq-all > gpurun_out/cert_timeline.md
echo done
